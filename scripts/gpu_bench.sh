#!/bin/bash
# One bench pass: the default bench line (+ optional Local / TTSD) into gpurun_out/bench/.
#   EXTRA="local ttsd" bash scripts/gpu_bench.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bench
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; if [ $rc -ne 0 ]; then tail -20 $O/bench.err; exit $rc; fi
for x in ${EXTRA:-}; do
  if [ $x = local ]; then A="--config local --steps 2 --warmup 1"; else A="--config ttsd --steps 1 --warmup 0 --no-cpu-baseline"; fi
  timeout -k 10 900 python -u bench.py $A > $O/bench_$x.json 2> $O/bench_$x.err
  rc=$?; echo "bench $x rc=$rc"; cat $O/bench_$x.json; if [ $rc -ne 0 ]; then tail -20 $O/bench_$x.err; exit $rc; fi
done
