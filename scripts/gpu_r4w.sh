#!/bin/bash
# Round 4 session W: batch-4 attention with double-buffered chunk loads (var adb) vs default, and the
# batch-4 launch's per-layer phase trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
VARIANTS="moss_tts_amd/lib/var/libmtts_adb.so" bash scripts/lib_ab.sh 2>&1 | grep "B=4"
timeout -k 10 300 python -u scripts/pse4_trace.py 8 181 > $O/pse4_trace.txt 2>&1
rc=$?; echo "pse4 trace rc=$rc"; grep -v Warn $O/pse4_trace.txt | tail -7
