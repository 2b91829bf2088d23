#!/bin/bash
# Round 4 session Q: gemm3's one-token-block form for <= 192-row prompts.  Packed GEMM parity at the
# 8B shapes, the packed-prefill engine test, then prefill times with the form on / off and the
# 181-row prefill's kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/tests.txt | tail -16; if [ $rc -ne 0 ]; then exit $rc; fi
for v in 12 0; do
  MTTS_GEMM3_SMALL=$v PREFILL_SHAPES=1x181,1x130,4x181,1x512 timeout -k 10 200 python3 scripts/prefill_probe.py > $O/p$v.txt 2>&1 || { tail -3 $O/p$v.txt; exit 1; }
  echo "GEMM3_SMALL=$v"; grep prefill $O/p$v.txt
done
PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pq -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o.txt 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
cp $(find /tmp/pq -name "*kernel_stats.csv" | head -1) $O/stats_1x181.csv
echo done
