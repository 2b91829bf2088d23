#!/bin/bash
# Same-box A/B of library builds (MTTS_LIB): for each lib in $LIBS (default build first) run each
# bench argument list of $BENCHES (';'-separated), $REPS times interleaved; prints key numbers.
#   LIBS="moss_tts_amd/lib/var/libmtts_base.so" BENCHES="--batch 1;--config local" bash scripts/ab_libs.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra LIST <<< "${BENCHES:---batch 1}"
for rep in $(seq 1 ${REPS:-2}); do
for lib in moss_tts_amd/lib/libmtts.so ${LIBS:-}; do
  for b in "${LIST[@]}"; do
    MTTS_LIB=$lib timeout -k 10 400 python3 bench.py $b --steps ${STEPS:-3} --no-cpu-baseline --no-codec --no-roofline --extra-batches "" > $O/r.json 2> $O/e.txt
    rc=$?; [ $rc -eq 0 ] || { echo "$lib '$b' rc=$rc"; tail -5 $O/e.txt; exit $rc; }
    python3 - "$O/r.json" "$lib" "$b" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["value", "ms_per_decode_step", "ms_per_frame", "prefill_ms", "p50_first_chunk_ms"]
print(sys.argv[2].split('/')[-1], sys.argv[3], {k: d[k] for k in keys if k in d}, flush=True)
PY
  done
done
done
