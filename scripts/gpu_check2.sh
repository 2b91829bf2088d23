#!/bin/bash
# GPU tests (all, or $TESTS) + smoke + a short default bench line.  Writes gpurun_out/check/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -4 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
exit $rc
