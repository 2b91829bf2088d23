#!/bin/bash
# PMC of whole TTSD decode steps with a per-kernel split (separate FETCH_SIZE / WRITE_SIZE passes).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_CONFIGS="ttsd" bash scripts/pmc_round.sh
