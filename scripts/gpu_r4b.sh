#!/bin/bash
# Round 4 session B: evidence passes.  PMC traffic of the batch-4 launch and of whole TTSD decode
# steps (separate FETCH_SIZE / WRITE_SIZE passes), MFMA-busy of the prefill GEMMs, the B=1 prefill
# with gemm3 from 128 token rows vs the default, and a kernel trace of the B=4 bench.
# Writes gpurun_out/r4b/ and gpurun_out/pmc/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
PMC_CONFIGS="${PMC_CONFIGS:-pse4 ttsd}" bash scripts/pmc_round.sh || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/mfma -o m \
    --output-format csv -- python3 scripts/mfma_probe.py > $O/mfma_probe.json 2> $O/mfma_probe.err
rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/mfma_probe.err; exit $rc; }
python3 scripts/mfma_probe.py --summarize /tmp/mfma > $O/pmc_mfma.json && cat $O/pmc_mfma.json
for g3 in 512 128; do
  MTTS_GEMM3_MIN=$g3 timeout -k 10 300 python3 bench.py --batch 1 --steps 2 --warmup 1 --no-cpu-baseline --no-codec \
      --no-dp-leg --no-roofline --extra-batches "" > $O/b1_g3_$g3.json 2> $O/b1_g3_$g3.err
  rc=$?; [ $rc -eq 0 ] || { echo "b1 g3=$g3 rc=$rc"; tail -5 $O/b1_g3_$g3.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/b1_g3_$g3.json')); print('B=1 gemm3_min=$g3', {k: d[k] for k in ('value','prefill_ms','ms_per_decode_step')})"
done
BATCH=4 bash scripts/prof_batch.sh
