#!/bin/bash
# Round 4 session Y: what bounds gemm3's <= 192-row form -- kernel times at 181 rows with every k
# step re-reading activation k tile 0 (var px) or weight k tile 0 (var pw) vs the real build
# (timing probes only: their outputs are wrong by construction).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4y
mkdir -p $O
for v in base px pw; do
  lib=moss_tts_amd/lib/libmtts.so; [ $v != base ] && lib=moss_tts_amd/lib/var/libmtts_$v.so
  MTTS_LIB=$lib PREFILL_SHAPES=1x181 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/py_$v -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o_$v.txt 2> $O/e_$v.txt || { tail -3 $O/e_$v.txt; exit 1; }
  cp $(find /tmp/py_$v -name "*kernel_stats.csv" | head -1) $O/stats_$v.csv
  echo "== $v"; grep prefill $O/o_$v.txt; grep gemm3 $O/stats_$v.csv | cut -d, -f1-4
done
