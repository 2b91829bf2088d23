#!/bin/bash
# One GPU session of named steps: scripts/gpu_steps.sh OUTDIR SECONDS "cmd" [SECONDS "cmd" ...]
# Each step runs under its own `timeout -k 10`, writes gpurun_out/OUTDIR/stepN.log, and the
# session stops at the first failing step (no GPU work after a fault, an abort or a timeout).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
i=0
while [ $# -ge 2 ]; do
  lim=$1; cmd=$2; shift 2
  i=$((i + 1))
  start=$(date +%s)
  echo "step $i: $cmd" | tee -a "$O/steps.txt"
  timeout -k 10 "$lim" bash -c "$cmd" > "$O/step$i.log" 2>&1
  rc=$?
  echo "step $i rc=$rc in $(( $(date +%s) - start )) s" | tee -a "$O/steps.txt"
  tail -4 "$O/step$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
