#!/bin/bash
# Round 4 session V: PMC HBM traffic of the batch-1 / batch-4 persistent launches and the TTSD step
# after the attention callee-saved fix (separate FETCH_SIZE / WRITE_SIZE passes).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_CONFIGS="pse pse4 ttsd" bash scripts/pmc_round.sh
