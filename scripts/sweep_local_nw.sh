#!/bin/bash
# MossTTSLocal frame time vs forced waves-per-block (MTTS_NW="qkv,o,gu,down,heads"; 0 = auto)
cd "$GRAFT_REPO_ROOT"
for nw in "0,0,0,0,0" "8,0,0,0,0" "16,0,0,0,0" "0,4,0,0,0" "0,16,0,0,0" "0,0,8,0,0" "0,0,16,0,0" "0,0,0,4,0" "0,0,0,8,0"; do
  r=$(MTTS_NW=$nw timeout -k 10 120 python bench.py --config local --steps 1 --warmup 1 --decode-steps 40 --no-cpu-baseline 2>/dev/null)
  rc=$?
  if [ $rc -ne 0 ]; then echo "nw=$nw rc=$rc"; exit $rc; fi
  echo "nw=$nw $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_frame"], d["roofline"]["avg_launch_us"])')"
done
