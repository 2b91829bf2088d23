#!/bin/bash
# Round 4 session AA: gemm5 k steps in flight (MTTS_GEMM5 = 4 / 6 / 8): packed GEMM parity at 6 and 8,
# prefill times.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
for g in 6 8; do
  MTTS_GEMM5=$g timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "packed" > $O/tests_$g.txt 2>&1
  rc=$?; echo "tests R=$g rc=$rc"; tail -1 $O/tests_$g.txt; if [ $rc -ne 0 ]; then exit $rc; fi
done
for rep in 1 2; do
for g in 4 6 8; do
  MTTS_GEMM5=$g PREFILL_SHAPES=1x181,1x130 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "R=$g"; grep prefill $O/p.txt
done
done
