#!/bin/bash
# Same-box A/B of engine env settings: for each setting in $ENVS (';'-separated) run each bench
# argument list of $BENCHES (';'-separated), $REPS times interleaved; prints key numbers.
#   ENVS="MTTS_NONE=1;MTTS_ATTN_SPEC=0" BENCHES="--batch 1;--config local" bash scripts/ab_env.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra ELIST <<< "${ENVS:-MTTS_NONE=1}"
IFS=';' read -ra LIST <<< "${BENCHES:---batch 1}"
for rep in $(seq 1 ${REPS:-2}); do
for e in "${ELIST[@]}"; do
  for b in "${LIST[@]}"; do
    env $e timeout -k 10 400 python3 bench.py $b --steps ${STEPS:-3} --no-cpu-baseline --no-codec --no-roofline --extra-batches "" > $O/r.json 2> $O/e.txt
    rc=$?; [ $rc -eq 0 ] || { echo "$e '$b' rc=$rc"; tail -5 $O/e.txt; exit $rc; }
    python3 - "$O/r.json" "$e" "$b" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["value", "ms_per_decode_step", "ms_per_frame", "prefill_ms", "p50_first_chunk_ms"]
print(sys.argv[2], sys.argv[3], {k: d[k] for k in keys if k in d}, flush=True)
PY
  done
done
done
