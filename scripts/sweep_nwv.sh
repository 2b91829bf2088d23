#!/bin/bash
# decode attention waves per block (MTTS_ATTN_NWV) at B=1/4/16 and the Local config
cd "$GRAFT_REPO_ROOT"
for v in 8 16; do
  r=$(MTTS_ATTN_NWV=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --extra-batches 4,16 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "nwv=$v rc=$rc"; exit $rc; fi
  echo "delay nwv=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_decode_step"], d["value"], d["batch_sweep"])')"
  r=$(MTTS_ATTN_NWV=$v timeout -k 10 200 python bench.py --config local --steps 1 --warmup 1 --decode-steps 40 --no-cpu-baseline 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "local nwv=$v rc=$rc"; exit $rc; fi
  echo "local nwv=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_frame"], d["value"])')"
done
