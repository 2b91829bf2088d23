# persistent decode launch: parity tests, per-stage trace, then a short A/B bench
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mega_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mega_test.log 2>&1
rc=$?; echo "mega pytest rc=$rc"; tail -8 gpurun_out/mega_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/mega_trace.py > gpurun_out/mega_trace.txt 2>&1 || { echo "trace failed"; tail -20 gpurun_out/mega_trace.txt; exit 1; }
cat gpurun_out/mega_trace.txt
if [ "${BENCH:-1}" = 1 ]; then
for m in 1 0; do
  MTTS_MEGA=$m timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --extra-batches 2 > gpurun_out/bench_mega$m.json 2> gpurun_out/bench_mega$m.err || { echo "bench mega=$m failed"; tail -5 gpurun_out/bench_mega$m.err; exit 1; }
  echo "MEGA=$m"; python -c "import json,sys; d=json.loads(open('gpurun_out/bench_mega$m.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_decode_step'], d.get('batch_sweep'))"
done
fi
