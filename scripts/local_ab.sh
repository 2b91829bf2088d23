#!/bin/bash
# Local frame A/B of one engine switch: the Local GPU tests, then the Local bench with the
# default and with $AB_ENV set (same box).  Writes gpurun_out/lab/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_local_gpu.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for side in a b a b; do
  if [ $side = b ]; then E="$AB_ENV"; else E="MTTS_NONE=1"; fi
  env $E timeout -k 10 400 python3 bench.py --config local --steps 3 --warmup 1 --no-cpu-baseline > $O/$side.json 2> $O/$side.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $side rc=$rc"; tail -5 $O/$side.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$O/$side.json')); print('$side', '$E', d['value'], d.get('ms_per_frame'), d['roofline']['frac'])"
done
