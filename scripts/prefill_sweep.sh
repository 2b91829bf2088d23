#!/bin/bash
# Prefill timing: MTTS_GEMM3_SMALL_MINK sweep for the 181-row clone prompt, then rocprofv3 kernel
# stats of the clone (1x181) and TTSD (1x2117, one chunk) prefills.  Writes gpurun_out/pf/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pf
mkdir -p $O
for mk in 8 16 32; do
  MTTS_GEMM3_SMALL_MINK=$mk PREFILL_SHAPES=1x181,4x181 timeout -k 10 200 python3 scripts/prefill_probe.py > $O/mink$mk.txt 2>&1 || { tail -3 $O/mink$mk.txt; exit 1; }
  echo "mink=$mk: $(grep prefill $O/mink$mk.txt | tr '\n' ' ')"
done
for sh in 1x181 1x2117; do
  PREFILL_SHAPES=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pf_$sh -o run --output-format csv -- python3 scripts/prefill_probe.py > $O/prof_$sh.txt 2> $O/prof_$sh.err || { tail -3 $O/prof_$sh.err; exit 1; }
  cp $(find /tmp/pf_$sh -name "*kernel_stats.csv" | head -1) $O/stats_$sh.csv
  echo "== $sh: $(grep prefill $O/prof_$sh.txt)"; python3 scripts/kstats.py $O/stats_$sh.csv 14
done
