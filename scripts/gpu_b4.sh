#!/bin/bash
# Batch-4 persistent launch (pse4.hip): parity tests, then B=4 bench lines with the launch on / off.
# Writes gpurun_out/b4/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/b4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_b4_oracle_gpu.py} -m gpu -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED|REFIDS" $O/pytest.log | tail -40; tail -3 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for flag in 1 0; do
  MTTS_PSE4=$flag timeout -k 10 300 python -u bench.py --batch 4 --steps 3 --warmup 1 --no-cpu-baseline --no-codec \
      --no-dp-leg --extra-batches "" > $O/bench_b4_pse$flag.json 2> $O/bench_b4_pse$flag.err
  rc=$?; echo "bench pse4=$flag rc=$rc"; cat $O/bench_b4_pse$flag.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: d.get(k) for k in ('value','ms_per_decode_step','decode_step_hbm_frac','prefill_ms')}, d['roofline'] and {k: d['roofline'].get(k) for k in ('frac','avg_launch_us','kernel')})"
  if [ $rc -ne 0 ]; then tail -5 $O/bench_b4_pse$flag.err; exit $rc; fi
done
