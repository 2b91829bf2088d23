#!/bin/bash
# Round 4 session E: the counter form of the residual hand-offs in the batch-1 launch (PSE_HCNT):
# the launch's parity tests on that build, then B=1 bench lines default / PSE_HCNT (2 reps each,
# interleaved).  Writes gpurun_out/r4e/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
V=moss_tts_amd/lib/var/libmtts_phcnt.so
MTTS_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_pse_gpu.py tests/test_pse_oracle_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_phcnt.log 2>&1
rc=$?; echo "pse tests (phcnt lib) rc=$rc"; tail -3 $O/pytest_phcnt.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in moss_tts_amd/lib/libmtts.so $V ${EXTRA_LIBS:-}; do
    MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
        --extra-batches "" > $O/b1.json 2> $O/b1.err
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b1.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/b1.json')); r=d['roofline']; print('$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')}, r['frac'], r['avg_launch_us'])"
  done
done
