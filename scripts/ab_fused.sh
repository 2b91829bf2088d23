#!/bin/bash
# A/B: fused decode attention + o_proj (default) vs two launches (MTTS_FUSED_AO=0)
cd "$GRAFT_REPO_ROOT"
for v in 1 0; do
  r=$(MTTS_FUSED_AO=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extra-batches 4,16 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "fused=$v rc=$rc"; exit $rc; fi
  echo "delay fused=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_decode_step"], d["value"], d["batch_sweep"])')"
  r=$(MTTS_FUSED_AO=$v timeout -k 10 200 python bench.py --config local --steps 1 --warmup 1 --decode-steps 40 --no-cpu-baseline 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "local fused=$v rc=$rc"; exit $rc; fi
  echo "local fused=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_frame"], d["value"])')"
done
