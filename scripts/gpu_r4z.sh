#!/bin/bash
# Round 4 session Z: the split-path <= 192-row GEMM (gemm5: weights by LDS-DMA, activations straight
# to VGPRs) vs gemm3's form (MTTS_GEMM5=0): packed GEMM + engine parity, prefill times, kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" $O/tests.txt; grep -E "FAIL|Error" $O/tests.txt | tail -5; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for g in 1 0; do
  MTTS_GEMM5=$g PREFILL_SHAPES=1x181,1x130,2x90 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "MTTS_GEMM5=$g"; grep prefill $O/p.txt
done
done
PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pz -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o.txt 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
cp $(find /tmp/pz -name "*kernel_stats.csv" | head -1) $O/stats_1x181.csv
grep gemm $O/stats_1x181.csv | cut -d, -f1-4
