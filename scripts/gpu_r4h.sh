#!/bin/bash
# Round 4 session H: batch-4 launch with release-flag hand-offs for h and the attention output (the
# new default) -- parity tests, trace, A/B against the h-only build; then the evidence passes of
# session B (PMC pse4 / ttsd, MFMA busy, B=1 gemm3 A/B, B=4 kernel trace) and the TTSD timelines.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_b4_oracle_gpu.py tests/test_pse_gpu.py -m gpu -q -p no:cacheprovider \
    --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "b4 + pse tests rc=$rc"; tail -2 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/pse4_trace.py 8 181 > $O/pse4_trace.txt 2>&1
rc=$?; echo "trace rc=$rc"; grep -v Warn $O/pse4_trace.txt | tail -8; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in moss_tts_amd/lib/libmtts.so moss_tts_amd/lib/var/libmtts_attf0.so; do
    MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --batch 4 --steps 2 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
        --extra-batches "" > $O/b4.json 2> $O/b4.err
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b4.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/b4.json')); r=d['roofline']; print('B=4', '$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')}, r['frac'], r['avg_launch_us'])"
  done
done
bash scripts/gpu_r4b.sh || exit $?
TEXT_TOKENS="2000 8000" DSTEPS=48 bash scripts/prof_longctx.sh
