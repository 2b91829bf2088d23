#!/bin/bash
# Round 4 session U: gemm4 (register-staged loads) vs gemm3 (LDS-DMA): GEMM / packed-prefill parity,
# prefill times per MTTS_GEMM4 setting, kernel stats of the 181-row prefill, MFMA-busy pass.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" $O/tests.txt; grep -E "FAIL|Error" $O/tests.txt | tail -5; if [ $rc -ne 0 ]; then exit $rc; fi
for g in 3 0 1 2; do
  MTTS_GEMM4=$g PREFILL_SHAPES=1x181,4x181,1x1024,1x2048,32x181 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "MTTS_GEMM4=$g"; grep prefill $O/p.txt
done
PREFILL_SHAPES=1x2100 PREFILL_MAXCTX=9700 PREFILL_CHUNK=1024 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/pt.txt 2>&1 || { tail -3 $O/pt.txt; exit 1; }
echo "TTSD long form"; grep prefill $O/pt.txt
PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pu -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o.txt 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
cp $(find /tmp/pu -name "*kernel_stats.csv" | head -1) $O/stats_1x181.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pm -o m --output-format csv -- python3 scripts/mfma_probe.py > $O/m.txt 2>&1 || { tail -3 $O/m.txt; exit 1; }
python3 scripts/mfma_probe.py --summarize /tmp/pm > $O/pmc_mfma.json && grep -B1 -A1 "weighted" $O/pmc_mfma.json | grep -v "^--" | paste - - - | sed 's/ \+/ /g'
echo done
