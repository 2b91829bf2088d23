#!/bin/bash
# Prefill GEMM block-tile sweep (MTTS_GEMM_TILE 0: 128x128, 1: 128x64, 2: 64x128, 3: 64x64):
# x split-K (MTTS_GEMM_SPLITK -1: auto, 0: off, S: forced); B=1 clone prefill ms, B=32 prefill ms.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gt
for t in ${TILES:-0 1 2 3}; do for sk in ${SPLITS:--1}; do
  for b in 1 32; do
    MTTS_GEMM_SPLITK=$sk MTTS_GEMM_TILE=$t timeout -k 10 300 python bench.py --batch $b --steps 1 --warmup 1 --no-cpu-baseline --no-codec --no-roofline --extra-batches "" > gpurun_out/gt/r.json 2> gpurun_out/gt/e.txt || { tail -3 gpurun_out/gt/e.txt; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/gt/r.json'));print('tile=$t sk=$sk B=$b prefill_ms', d['prefill_ms'], 'value', d['value'])"
  done
done
done
