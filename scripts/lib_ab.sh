#!/bin/bash
# Bench the default build against library variants (MTTS_LIB): B=1 and B=4 decode step times.
#   VARIANTS="moss_tts_amd/lib/var/libmtts_v1.so ..." bash scripts/lib_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lib_ab
for rep in 1 2; do
for lib in moss_tts_amd/lib/libmtts.so ${VARIANTS:-}; do
  for b in 1 4; do
    MTTS_LIB=$lib timeout -k 10 300 python bench.py --batch $b --steps 3 --no-cpu-baseline --no-codec --no-roofline --extra-batches "" > gpurun_out/lib_ab/r.json 2> gpurun_out/lib_ab/e.txt || { tail -3 gpurun_out/lib_ab/e.txt; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/lib_ab/r.json'));print('$lib B=$b', d['value'], d['ms_per_decode_step'], 'prefill', d.get('prefill_ms'))"
  done
done
done
