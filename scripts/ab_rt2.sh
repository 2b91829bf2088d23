#!/bin/bash
# A/B: RT=2 plain projections from MTTS_GEMV_RT2 rows (default 8) vs off (0)
cd "$GRAFT_REPO_ROOT"
for v in 12 0; do
  r=$(MTTS_GEMV_RT2=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --extra-batches 8,16,32 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "rt2=$v rc=$rc"; exit $rc; fi
  echo "delay rt2=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_decode_step"], d["value"], d["batch_sweep"])')"
  r=$(MTTS_GEMV_RT2=$v timeout -k 10 200 python bench.py --config local --steps 1 --warmup 1 --decode-steps 40 --no-cpu-baseline 2>/dev/null)
  rc=$?; if [ $rc -ne 0 ]; then echo "local rt2=$v rc=$rc"; exit $rc; fi
  echo "local rt2=$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_frame"], d["value"])')"
done

