#!/bin/bash
# B=32 decode: GEMV NW for 17-32 rows, GEMM path for the projections, attention waves
cd "$GRAFT_REPO_ROOT"
run() {
  r=$(env "$@" timeout -k 10 200 python bench.py --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --extra-batches "" --no-roofline 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "$* rc=$rc"; exit $rc; fi
  echo "$* $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_decode_step"], d["value"])')"
}
run X=0
run MTTS_GEMM_MIN_ROWS=17
run MTTS_NW=8,8,8,8,0
run MTTS_NW=16,16,0,16,0
run MTTS_GEMV_PIPE=2
run MTTS_GEMV_PIPE=2 MTTS_NW=8,8,8,8,0
run MTTS_ATTN_NWV=16
