#!/bin/bash
# Per-kernel averages of the prefill for each library variant (MTTS_LIB), rocprofv3 kernel stats.
#   VARIANTS="moss_tts_amd/lib/var/libmtts_x.so ..." SHAPES=1x181 bash scripts/ab_prefill_prof.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab_prefill_prof
mkdir -p $O
i=0
for lib in moss_tts_amd/lib/libmtts.so ${VARIANTS:-}; do
  i=$((i + 1))
  MTTS_LIB=$lib PREFILL_SHAPES=${SHAPES:-1x181} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abp$i -o run \
      --output-format csv -- python3 scripts/prefill_probe.py > $O/run$i.txt 2>&1 || { tail -3 $O/run$i.txt; exit 1; }
  echo "== $lib: $(grep prefill $O/run$i.txt | tr '\n' ' ')" | tee -a $O/summary.txt
  python3 scripts/kstats.py $(find /tmp/abp$i -name "*kernel_stats.csv" | head -1) ${TOP:-6} | tee -a $O/summary.txt
done
