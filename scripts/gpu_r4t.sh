#!/bin/bash
# Round 4 session T: gemm3 shape sweeps -- 256-row blocks for every matrix (MTTS_GEMM3_WIDE=0), a
# 4-stage ring (var nst4), the small form's stage count (var snst5) and split depth (MINK 16).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
run() {  # label, env..., then shapes
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 scripts/prefill_probe.py > $O/p.txt 2>&1 || { tail -3 $O/p.txt; exit 1; }
  echo "$label"; grep prefill $O/p.txt
}
S=1x181,4x181,1x1024,1x2048,32x181
run default PREFILL_SHAPES=$S
run wide0 MTTS_GEMM3_WIDE=0 PREFILL_SHAPES=$S
run nst4 MTTS_LIB=moss_tts_amd/lib/var/libmtts_nst4.so PREFILL_SHAPES=$S
run snst5 MTTS_LIB=moss_tts_amd/lib/var/libmtts_snst5.so PREFILL_SHAPES=1x181,1x130
run smink16 MTTS_GEMM3_SMALL_MINK=16 PREFILL_SHAPES=1x181,1x130
run default2 PREFILL_SHAPES=$S
echo done
