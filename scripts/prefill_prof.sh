#!/bin/bash
# rocprofv3 kernel stats of B=1 prefills only (mtts_forward over the clone prompt, no decode)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
for t in ${TILES:-0 1}; do
  PREFILL_SHAPES=${SHAPES:-1x181} MTTS_GEMM_TILE=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ppf$t -o run --output-format csv -- python3 scripts/prefill_probe.py > gpurun_out/pp/o$t.txt 2> gpurun_out/pp/e$t.txt || { tail -3 gpurun_out/pp/e$t.txt; exit 1; }
  cp $(find /tmp/ppf$t -name "*kernel_stats.csv" | head -1) gpurun_out/pp/stats$t.csv
  echo "tile=$t"; cut -d, -f1-4 gpurun_out/pp/stats$t.csv | head -12
done
