#!/bin/bash
# Counter evidence on the HEAD kernels: PMC HBM traffic of the batch-1 persistent launch
# (separate FETCH_SIZE / WRITE_SIZE passes), MFMA-busy of the prefill GEMMs, and a B=4 decode
# step timeline.  Writes gpurun_out/evidence/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/evidence
mkdir -p $O
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace -d /tmp/pmc_pse -o ${c}_pse --output-format csv -- \
      python3 scripts/pmc_probe.py --config pse > $O/probe_pse_$c.json 2> $O/probe_pse_$c.err
  rc=$?; echo "pse $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/probe_pse_$c.err; exit $rc; fi
done
python3 scripts/pmc_probe.py --summarize /tmp/pmc_pse --config pse > $O/pmc_pse.json; cat $O/pmc_pse.json
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/pmc_mfma -o mfma \
    --output-format csv -- python3 scripts/mfma_probe.py > $O/mfma_probe.json 2> $O/mfma_probe.err
rc=$?; echo "mfma rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/mfma_probe.err; exit $rc; fi
python3 scripts/mfma_probe.py --summarize /tmp/pmc_mfma > $O/pmc_mfma.json; cat $O/pmc_mfma.json
cp $(find /tmp/pmc_mfma -name "*kernel_trace.csv" | head -1) $O/mfma_kernel_trace.csv
BATCH=4 SEQ=40 timeout -k 10 300 bash scripts/prof_batch.sh > $O/prof_b4.txt 2>&1
rc=$?; echo "prof b4 rc=$rc"; head -60 $O/prof_b4.txt
