#!/bin/bash
# gpurun with a wait for a free box: re-submits only while gpurun answers 3 (no box / slot free
# right now, nothing ran, nothing charged); any other exit -- including a failing GPU step --
# ends it.  Usage: scripts/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "gpurun rc=$rc" >> "$out"; exit $rc; fi
  sleep 90
done
