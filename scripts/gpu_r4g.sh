#!/bin/bash
# Round 4 session G: release-flag residual hand-offs (PSE_HCNT=2 / PSE4_HCNT=2) -- parity tests on
# those builds, then B=1 and B=4 bench lines default / variant, interleaved.  gpurun_out/r4g/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
V1=moss_tts_amd/lib/var/libmtts_phcnt2.so
V4=moss_tts_amd/lib/var/libmtts_hcnt2.so
MTTS_LIB=$V1 timeout -k 10 300 python -u -m pytest tests/test_pse_gpu.py tests/test_pse_oracle_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest_v1.log 2>&1
rc=$?; echo "pse tests ($V1) rc=$rc"; tail -2 $O/pytest_v1.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MTTS_LIB=$V4 timeout -k 10 300 python -u -m pytest tests/test_b4_oracle_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest_v4.log 2>&1
rc=$?; echo "b4 tests ($V4) rc=$rc"; tail -2 $O/pytest_v4.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in moss_tts_amd/lib/libmtts.so $V1; do
    MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
        --extra-batches "" > $O/b1.json 2> $O/b1.err
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b1.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/b1.json')); r=d['roofline']; print('B=1', '$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')}, r['frac'], r['avg_launch_us'])"
  done
  for lib in moss_tts_amd/lib/libmtts.so $V4; do
    MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --batch 4 --steps 2 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
        --extra-batches "" > $O/b4.json 2> $O/b4.err
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b4.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/b4.json')); r=d['roofline']; print('B=4', '$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')}, r['frac'], r['avg_launch_us'])"
  done
done
