#!/bin/bash
# One GPU session: smoke, parity tests, the default bench line (+ Local, TTSD), rocprofv3
# kernel-trace summaries of the default and Local benches.  Writes gpurun_out/round/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${ROUND_TAG:-round}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config local --steps 2 --warmup 1 > $O/bench_local.json 2> $O/bench_local.err
rc=$?; echo "bench local rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --config ttsd --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_ttsd.json 2> $O/bench_ttsd.err
rc=$?; echo "bench ttsd rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_d -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --extra-batches "" > $O/prof_bench.json 2> $O/prof.err
  rc=$?; echo "rocprof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  cp $(find /tmp/prof_d -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
  python3 scripts/ktrace.py $(find /tmp/prof_d -name "*kernel_trace.csv" | head -1) > $O/decode_step_timeline.txt
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_l -o run --output-format csv -- \
      python3 bench.py --config local --steps 1 --warmup 1 --decode-steps 24 --no-cpu-baseline > $O/prof_local.json 2> $O/prof_local.err
  rc=$?; echo "rocprof local rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
  cp $(find /tmp/prof_l -name "*kernel_stats.csv" | head -1) $O/local_kernel_stats.csv
  python3 scripts/ktrace_local.py $(find /tmp/prof_l -name "*kernel_trace.csv" | head -1) > $O/local_frame_timeline.txt
fi
