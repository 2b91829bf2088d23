#!/bin/bash
# In-context A/B of engine env toggles: each argument is "VAR=val[,VAR=val...]"; prints ms/step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "${@}"; do
  envs=$(echo "$cfg" | tr ',' ' ')
  r=$(env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --extra-batches "" --steps 2 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_decode_step'], d['prefill_ms'], d['value'])")
  rc=$?; echo "$cfg -> $r"; [ $rc -ne 0 ] && exit $rc
done
exit 0
