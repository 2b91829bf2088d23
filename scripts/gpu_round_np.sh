#!/bin/bash
# The round-end session without the rocprofv3 passes (smoke, GPU tests, bench lines)
PROFILE=0 bash "$GRAFT_REPO_ROOT/scripts/gpu_round.sh"
