#!/bin/bash
# rocprofv3 kernel trace of the default bench at one batch size: per-kernel stats + one decode step's timeline.
#   BATCH=32 bash scripts/prof_batch.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_b${BATCH:-32}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_b -o run --output-format csv -- \
    python3 bench.py --batch ${BATCH:-32} --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-codec --extra-batches "" > $O/bench.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof.err; exit $rc; }
cp $(find /tmp/prof_b -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
KTRACE_SEQ=${SEQ:-0} python3 scripts/ktrace.py $(find /tmp/prof_b -name "*kernel_trace.csv" | head -1) > $O/decode_step_timeline.txt
head -40 $O/decode_step_timeline.txt
