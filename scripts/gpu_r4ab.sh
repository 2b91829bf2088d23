#!/bin/bash
# Round 4 session AB: split paths for the long-prompt GEMM shapes too (MTTS_GEMM5_LONG=1) vs gemm3:
# packed GEMM + engine parity under both, prefill times, MFMA-busy pass with the switch on.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ab
mkdir -p $O
for g in 0 1; do
  MTTS_GEMM5_LONG=$g timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests_$g.txt 2>&1
  rc=$?; echo "tests LONG=$g rc=$rc"; tail -1 $O/tests_$g.txt; if [ $rc -ne 0 ]; then exit $rc; fi
done
for rep in 1 2; do
for g in 1 0; do
  MTTS_GEMM5_LONG=$g PREFILL_SHAPES=1x181,4x181,1x1024,1x2048,32x181 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "GEMM5_LONG=$g"; grep prefill $O/p.txt
done
done
MTTS_GEMM5_LONG=1 PREFILL_SHAPES=1x2100 PREFILL_MAXCTX=9700 PREFILL_CHUNK=1024 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/pt.txt 2>&1 || { tail -3 $O/pt.txt; exit 1; }
echo "TTSD long form, GEMM5_LONG=1"; grep prefill $O/pt.txt
