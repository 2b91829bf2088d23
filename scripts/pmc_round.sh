#!/bin/bash
# PMC traffic of the bench's dominant kernel (separate FETCH_SIZE / WRITE_SIZE passes)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for cfg in ${PMC_CONFIGS:-clone local}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d /tmp/pmc_$cfg -o ${c}_$cfg --output-format csv -- \
        python3 scripts/pmc_probe.py --config $cfg > gpurun_out/pmc/probe_${cfg}_$c.json 2> gpurun_out/pmc/probe_${cfg}_$c.err
    rc=$?; echo "$cfg $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/probe_${cfg}_$c.err; exit $rc; fi
  done
  python3 scripts/pmc_probe.py --summarize /tmp/pmc_$cfg --config $cfg > gpurun_out/pmc/pmc_$cfg.json
  cat gpurun_out/pmc/pmc_$cfg.json
done
