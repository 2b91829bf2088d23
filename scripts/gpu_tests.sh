#!/bin/bash
# GPU parity pass: smoke, then the -m gpu suite (optionally a subset: TESTS="tests/x.py ...").
# Writes gpurun_out/tests/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tests
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat $O/smoke.log | grep -v Warning | tail -25
# an assertion (rc 1) still lets the parity suite run; a crash / signal / timeout ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED" $O/pytest_gpu.log | tail -80; tail -3 $O/pytest_gpu.log
exit $rc
