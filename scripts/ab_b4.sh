#!/bin/bash
# Same-box A/B of library variants (MTTS_LIB) on the batch-4 decode step, interleaved reps.
#   VARIANTS="moss_tts_amd/lib/var/libmtts_x.so ..." REPS=3 BATCH=4 bash scripts/ab_b4.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_b4
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
for lib in moss_tts_amd/lib/libmtts.so ${VARIANTS:-}; do
  MTTS_LIB=$lib timeout -k 10 300 python bench.py --batch ${BATCH:-4} --steps 3 --warmup 1 --no-cpu-baseline --no-codec \
      --no-roofline --no-dp-leg --extra-batches "" > $O/r.json 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r.json'));print('$lib B=${BATCH:-4}', d['value'], d['ms_per_decode_step'], 'prefill', d.get('prefill_ms'))" | tee -a $O/summary.txt
done
done
