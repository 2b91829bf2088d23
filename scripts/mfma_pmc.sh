#!/bin/bash
# MFMA-busy counter passes for the prefill GEMMs / attention (scripts/mfma_probe.py), one per prompt
# shape: gpurun_out/mfma/pmc_mfma_<shape>.json
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mfma
mkdir -p $O
for sh in ${SHAPES:-b1 ttsd}; do
  MFMA_SHAPES=$sh timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pmc_mfma_$sh -o m \
      --output-format csv -- python3 scripts/mfma_probe.py > $O/probe_$sh.json 2> $O/probe_$sh.err
  rc=$?; echo "$sh rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/probe_$sh.err; exit $rc; fi
  python3 scripts/mfma_probe.py --summarize /tmp/pmc_mfma_$sh > $O/pmc_mfma_$sh.json && head -40 $O/pmc_mfma_$sh.json
done
