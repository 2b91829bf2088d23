#!/bin/bash
# Round 4 session R: gemm3 with a bare barrier (no vmcnt(0) per k step) and a uniform LDS-DMA
# destination.  GEMM parity, then prefill times: the small form on / off, gemm3 from 512 / 2,048 rows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" $O/tests.txt; grep -E "FAIL|Error" $O/tests.txt | tail -5; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests2.txt 2>&1
rc=$?; echo "engine packed tests rc=$rc"; grep -E "PASS|FAIL" $O/tests2.txt | tail -3; if [ $rc -ne 0 ]; then exit $rc; fi
for v in "12 2048" "0 2048" "12 512"; do
  set -- $v
  MTTS_GEMM3_SMALL=$1 MTTS_GEMM3_MIN=$2 PREFILL_SHAPES=1x181,1x130,4x181,1x1024,1x2048,32x181 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p_$1_$2.txt 2>&1 || { tail -3 $O/p_$1_$2.txt; exit 1; }
  echo "GEMM3_SMALL=$1 GEMM3_MIN=$2"; grep prefill $O/p_$1_$2.txt
done
PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pq -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o.txt 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
cp $(find /tmp/pq -name "*kernel_stats.csv" | head -1) $O/stats_1x181.csv
echo done
