#!/bin/bash
# In-context sweep of GEMV / attention launch shapes: the full decode bench under
# MTTS_NW="qkv,o,gu,down,heads" / MTTS_ATTN_NWV / MTTS_GEMV_PIPE overrides; cfg = nw/attn/pipe.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "${@}"; do
  IFS=/ read -r nw an pipe <<< "$cfg"
  r=$(MTTS_NW="$nw" MTTS_ATTN_NWV="$an" MTTS_GEMV_PIPE="${pipe:-0}" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_decode_step'], d['value'])")
  rc=$?; echo "MTTS_NW=$nw ATTN_NWV=$an PIPE=${pipe:-0} -> $r"; [ $rc -ne 0 ] && exit $rc
done
exit 0
