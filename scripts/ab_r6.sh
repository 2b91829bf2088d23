#!/bin/bash
# Round-6 A/B session: the batch-1 launch's warmer wave (PSE_WARM variants, MTTS_LIB) and the
# MossTTSLocal resident depth layers (MTTS_LOCAL_RESIDENT).  Writes gpurun_out/ab_r6/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_r6
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${WARM:-}" ]; then
  MTTS_LIB=moss_tts_amd/lib/var/libmtts_w16.so timeout -k 10 300 python -c "import __graft_entry__ as g; g._smoke_pse()" || exit 1
  VARIANTS="$WARM" REPS=2 BATCH=1 bash scripts/ab_b4.sh || exit 1
fi
for rep in 1 2; do
  for r in ${RESIDENT:-0 1 2}; do
    MTTS_LOCAL_RESIDENT=$r timeout -k 10 300 python bench.py --config local --steps 2 --warmup 1 --no-cpu-baseline \
        > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/l.json'));print('resident $r', d['ms_per_frame'], 'ms/frame', d['value'])" | tee -a $O/summary.txt
  done
done
