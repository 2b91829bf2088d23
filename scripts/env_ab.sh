#!/bin/bash
# Bench one batch size under several engine env settings (same box, same build):
#   BATCH=32 ENVS="MTTS_NONE=1;MTTS_GEMM_MIN_ROWS=17;MTTS_NW=8,8,8,8,8" bash scripts/env_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/env_ab
mkdir -p $O
IFS=';' read -ra LIST <<< "${ENVS:-MTTS_NONE=1}"
for rep in 1 2; do
for e in "${LIST[@]}"; do
  env $e timeout -k 10 300 python bench.py --batch ${BATCH:-32} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-codec --no-roofline --extra-batches "" > $O/r.json 2> $O/e.txt || { echo "FAILED: $e"; tail -3 $O/e.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r.json'));print('$e', 'B=${BATCH:-32}', d['value'], d['ms_per_decode_step'], 'prefill', d.get('prefill_ms'))"
done
done
