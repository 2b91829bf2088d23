#!/bin/bash
# B=32 decode sweep: cfg = MTTS_NW/MTTS_GEMV_PIPE
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "${@}"; do
  IFS=/ read -r nw pipe <<< "$cfg"
  r=$(MTTS_NW="$nw" MTTS_GEMV_PIPE="${pipe:-0}" timeout -k 10 300 python bench.py --batch 32 --no-cpu-baseline --no-roofline --extra-batches "" --steps 1 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_decode_step'], d['prefill_ms'], d['value'])")
  rc=$?; echo "B32 MTTS_NW=$nw PIPE=${pipe:-0} -> $r"; [ $rc -ne 0 ] && exit $rc
done
exit 0
