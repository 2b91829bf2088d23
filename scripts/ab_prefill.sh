#!/bin/bash
# Same-box A/B of library variants (MTTS_LIB) on prefill timings, interleaved reps.
#   VARIANTS="moss_tts_amd/lib/var/libmtts_x.so ..." SHAPES=1x181,1x2117 REPS=3 bash scripts/ab_prefill.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_prefill
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
for lib in moss_tts_amd/lib/libmtts.so ${VARIANTS:-}; do
  MTTS_LIB=$lib PREFILL_SHAPES=${SHAPES:-1x181,1x2117} timeout -k 10 200 python3 scripts/prefill_probe.py > $O/r.txt 2>&1 || { tail -3 $O/r.txt; exit 1; }
  echo "$lib: $(grep prefill $O/r.txt | tr '\n' ' ')" | tee -a $O/summary.txt
done
done
