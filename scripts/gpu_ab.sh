#!/bin/bash
# A/B of one engine switch on the GPU box: the given tests, the default bench with the switch
# on (env as given) and off (OFF_ENV), and a rocprofv3 kernel-trace timeline of one decode step.
#   TESTS="tests/test_pse_gpu.py" ON_ENV="MTTS_PSE=1" OFF_ENV="MTTS_PSE=0" bash scripts/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
B="${BENCH_ARGS:---no-cpu-baseline --extra-batches 4}"
env ${ON_ENV:-MTTS_NONE=1} timeout -k 10 300 python bench.py $B > $O/bench_on.json 2> $O/bench_on.err
rc=$?; echo "bench on rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_on.json'));print('ON ', d['value'], d['ms_per_decode_step'], d.get('batch_sweep'))"
[ $rc -eq 0 ] || exit $rc
env ${OFF_ENV:-MTTS_NONE=1} timeout -k 10 300 python bench.py $B > $O/bench_off.json 2> $O/bench_off.err
rc=$?; echo "bench off rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_off.json'));print('OFF', d['value'], d['ms_per_decode_step'], d.get('batch_sweep'))"
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  env ${ON_ENV:-MTTS_NONE=1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ab -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --extra-batches "" > $O/prof_bench.json 2> $O/prof.err
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp $(find /tmp/prof_ab -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
  python3 scripts/ktrace.py $(find /tmp/prof_ab -name "*kernel_trace.csv" | head -1) > $O/decode_step_timeline.txt
  head -20 $O/decode_step_timeline.txt
fi
