#!/bin/bash
# Round 4 session X: the <= 192-row gemm3 form with 2 k tiles per stage (MTTS_GEMM3_KD=2, 4 stages)
# vs 1 (5 stages): packed GEMM parity under both, prefill times.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
for kd in 1 2; do
  MTTS_GEMM3_KD=$kd timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "packed" > $O/tests_$kd.txt 2>&1
  rc=$?; echo "tests KD=$kd rc=$rc"; tail -1 $O/tests_$kd.txt; if [ $rc -ne 0 ]; then exit $rc; fi
done
for rep in 1 2; do
for kd in 1 2; do
  MTTS_GEMM3_KD=$kd PREFILL_SHAPES=1x181,1x130,2x90 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "KD=$kd"; grep prefill $O/p.txt
done
done
