#!/bin/bash
# Round 4 session S: gemm3 k order rotated per block (vs moss_tts_amd/lib/var/libmtts_norot.so), gemm3
# from 512 rows, the 4-lane split-K reduce.  GEMM / attention / packed-prefill parity, prefill times
# (B=1 181, B=4 181, 1,024, 2,048, B=32, TTSD long form), kernel stats of the 181-row prefill, and
# the MFMA-busy counter pass of scripts/mfma_probe.py.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or attention" "tests/test_engine_gpu.py::test_packed_activations_long_prefill" > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" $O/tests.txt; grep -E "FAIL|Error" $O/tests.txt | tail -5; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in moss_tts_amd/lib/libmtts.so moss_tts_amd/lib/var/libmtts_norot.so; do
  MTTS_LIB=$lib PREFILL_SHAPES=1x181,4x181,1x1024,1x2048,32x181 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "$lib"; grep prefill $O/p.txt
done
PREFILL_SHAPES=1x2100 PREFILL_MAXCTX=9700 PREFILL_CHUNK=1024 timeout -k 10 300 python3 scripts/prefill_probe.py > $O/pt.txt 2>&1 || { tail -3 $O/pt.txt; exit 1; }
echo "TTSD long form"; grep prefill $O/pt.txt
PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ps -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o.txt 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
cp $(find /tmp/ps -name "*kernel_stats.csv" | head -1) $O/stats_1x181.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pm -o m --output-format csv -- python3 scripts/mfma_probe.py > $O/m.txt 2>&1 || { tail -3 $O/m.txt; exit 1; }
python3 scripts/mfma_probe.py --summarize /tmp/pm > $O/pmc_mfma.json && tail -30 $O/pmc_mfma.json
echo done
