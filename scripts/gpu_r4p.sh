#!/bin/bash
# Round 4 session P: kernel stats of the batch-1 clone prefill (181 tokens) and a 2,048-token prefill.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
for sh in 1x181 1x2048; do
  PREFILL_SHAPES=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp_$sh -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/o_$sh.txt 2> $O/e_$sh.txt || { tail -3 $O/e_$sh.txt; exit 1; }
  cp $(find /tmp/pp_$sh -name "*kernel_stats.csv" | head -1) $O/stats_$sh.csv
  cp $(find /tmp/pp_$sh -name "*kernel_trace.csv" | head -1) $O/trace_$sh.csv
  cat $O/o_$sh.txt | grep prefill; cut -d, -f1-5 $O/stats_$sh.csv | head -16
done
