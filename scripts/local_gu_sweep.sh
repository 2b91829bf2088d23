#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for e in "MTTS_NONE=1" "MTTS_NW=0,0,8,0,0" "MTTS_NW=0,0,16,0,0" "MTTS_U=0,0,4,0,0" "MTTS_NW=0,0,8,0,0 MTTS_U=0,0,4,0,0" "MTTS_NO_NORM_DMA=1" "MTTS_NO_PRELOAD=1"; do
  r=$(env $e timeout -k 10 120 python3 scripts/pmc_probe.py --config local --iters 50 2>/dev/null | tail -1)
  echo "$e $r"
done
