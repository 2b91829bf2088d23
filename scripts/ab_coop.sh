#!/bin/bash
# Same-box A/B of the persistent launches' cooperative form (MTTS_PSE_COOP=1: hipLaunchCooperativeKernel,
# the runtime refuses a grid that cannot be co-resident) against the ordinary launch, B = 1 and 4.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_coop
mkdir -p $O
for rep in 1 2 3; do
  for coop in 0 1; do
    for b in 1 4; do
      MTTS_PSE_COOP=$coop timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-codec \
          --no-roofline --no-dp-leg --extra-batches "" > $O/r.json 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
      python3 -c "import json;d=json.load(open('$O/r.json'));print('coop $coop B=$b', d['value'], d['ms_per_decode_step'])" | tee -a $O/summary.txt
    done
  done
done
