#!/bin/bash
# Round-6 closing profiles: rocprofv3 kernel stats + step timelines of the B=1 bench (no dp leg, so the
# timeline's step is a batch-1 step) and the Local frame; PMC traffic passes of the batch-1 / batch-4
# launches and the TTSD step.  Writes gpurun_out/r06_g/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${ROUND_TAG:-r06_s}
mkdir -p $O gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_d -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dp-leg --no-codec --extra-batches "" > $O/prof_bench.json 2> $O/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp $(find /tmp/prof_d -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python3 scripts/ktrace.py $(find /tmp/prof_d -name "*kernel_trace.csv" | head -1) > $O/decode_step_timeline.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_l -o run --output-format csv -- \
    python3 bench.py --config local --steps 1 --warmup 1 --decode-steps 24 --no-cpu-baseline > $O/prof_local.json 2> $O/prof_local.err
rc=$?; echo "rocprof local rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp $(find /tmp/prof_l -name "*kernel_stats.csv" | head -1) $O/local_kernel_stats.csv
python3 scripts/ktrace_local.py $(find /tmp/prof_l -name "*kernel_trace.csv" | head -1) > $O/local_frame_timeline.txt
true
