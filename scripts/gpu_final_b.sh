#!/bin/bash
# Round-end evidence: PMC traffic of the bench's roofline kernels (separate FETCH_SIZE / WRITE_SIZE
# passes) and the batch-4 kernel timeline.  gpurun_out/pmc/, gpurun_out/prof_b4/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_CONFIGS="pse pse4 ttsd" bash scripts/pmc_round.sh || exit $?
BATCH=4 bash scripts/prof_batch.sh
