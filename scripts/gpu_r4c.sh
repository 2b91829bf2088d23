#!/bin/bash
# Round 4 session C: the MossTTSLocal persistent channel launch (lpse.hip) -- the B=8 parity tests on
# both paths, then the Local bench with the launch on / off.  Writes gpurun_out/r4c/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_local_b8_gpu.py ${EXTRA_TESTS:-} -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED" $O/pytest.log | tail -30; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
grep -E "^E " $O/pytest.log | head -20
for flag in 1 0; do
  MTTS_LPSE=$flag timeout -k 10 300 python3 bench.py --config local --steps 2 --warmup 1 --no-cpu-baseline \
      > $O/local_lpse$flag.json 2> $O/local_lpse$flag.err
  rc=$?; [ $rc -eq 0 ] || { echo "local lpse=$flag rc=$rc"; tail -5 $O/local_lpse$flag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/local_lpse$flag.json')); print('local lpse=$flag', {k: d.get(k) for k in ('value','ms_per_frame','frame_hbm_frac','prefill_ms')})"
done
