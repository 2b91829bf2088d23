#!/bin/bash
# prefill-only timings (scripts/prefill_probe.py) under several env settings
set -u
cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra LIST <<< "${ENVS:-MTTS_NONE=1}"
for e in "${LIST[@]}"; do
  echo "== $e"
  env $e PREFILL_SHAPES=${SHAPES:-1x181,1x512,4x181,1x100} timeout -k 10 200 python3 scripts/prefill_probe.py 2>/dev/null || { echo "FAILED $e"; exit 1; }
done
