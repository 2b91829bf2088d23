#!/bin/bash
# Round 4 session I: evidence passes (session B: PMC pse4 + ttsd, MFMA busy, B=1 gemm3 A/B, B=4 kernel
# trace) and the TTSD decode timelines at 2 K / 8 K contexts.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r4b.sh || exit $?
TEXT_TOKENS="2000 8000" DSTEPS=48 bash scripts/prof_longctx.sh
