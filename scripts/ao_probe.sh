#!/bin/bash
# attn_o_kernel duration under each timing probe (MTTS_AO_PROBE): rocprofv3 kernel stats of a
# short bench run per mode.  Results of probe runs are invalid by construction.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ao_probe
mkdir -p $O
export TMPDIR=/tmp
export MTTS_AO=1
for m in ${MODES:-0 1 2 3}; do
  MTTS_AO_PROBE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp$m -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --decode-steps 64 --no-cpu-baseline --no-roofline --no-codec --extra-batches "" > $O/b$m.json 2> $O/e$m.txt
  rc=$?; [ $rc -eq 0 ] || { echo "probe $m rc=$rc"; tail -5 $O/e$m.txt; exit $rc; }
  f=$(find /tmp/pp$m -name "*kernel_stats.csv" | head -1)
  cp $f $O/stats$m.csv
  echo "probe $m: $(grep -E 'attn_o_kernel|attn_decode_kernel' $f | cut -d, -f1-6 | tr '\n' ' ')"
done
