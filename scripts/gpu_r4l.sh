#!/bin/bash
# Round 4 session L: batch-4 launch trace with attention stamps; batch-1 trace (36 layers).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/pse4_trace.py 8 181 > $O/pse4_trace.txt 2>&1
rc=$?; echo "pse4 trace rc=$rc"; grep -v Warn $O/pse4_trace.txt | tail -7; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/pse_trace.py 36 181 > $O/pse_trace.txt 2>&1
rc=$?; echo "pse trace rc=$rc"; grep -v Warn $O/pse_trace.txt | tail -14
