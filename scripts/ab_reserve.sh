#!/bin/bash
# Round 6: reserve waves in the persistent launches (PSE_SW / PSE4_SW).  Parity of the default build
# (the reserve form) on the launch's GPU tests, then same-box interleaved A/B against variants.
#   VARIANTS="moss_tts_amd/lib/var/libmtts_sw0.so ..." BATCH=1 TESTS="tests/test_pse_gpu.py ..." bash scripts/ab_reserve.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_reserve
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for b in ${BATCH:-1}; do
  VARIANTS="${VARIANTS:-}" REPS=${REPS:-2} BATCH=$b bash scripts/ab_b4.sh || exit 1
done
