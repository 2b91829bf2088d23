#!/bin/bash
# Round 4 session F: the Local channel launch with release flags (LPSE_GO) -- B=8 tests, trace,
# Local bench lpse on / off / counter-polling build; then session E (batch-1 PSE_HCNT).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_local_b8_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "local tests rc=$rc"; tail -3 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/lpse_trace.py > $O/lpse_trace.txt 2>&1
rc=$?; echo "trace rc=$rc"; grep -v Warn $O/lpse_trace.txt | tail -12; if [ $rc -ne 0 ]; then exit $rc; fi
for v in "1 moss_tts_amd/lib/libmtts.so" "1 moss_tts_amd/lib/var/libmtts_lgo0.so" "0 moss_tts_amd/lib/libmtts.so"; do
  set -- $v
  MTTS_LPSE=$1 MTTS_LIB=$2 timeout -k 10 300 python3 bench.py --config local --steps 2 --warmup 1 --no-cpu-baseline \
      > $O/local.json 2> $O/local.err
  rc=$?; [ $rc -eq 0 ] || { echo "local $v rc=$rc"; tail -5 $O/local.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/local.json')); print('local lpse=$1 $(basename $2)', {k: d.get(k) for k in ('value','ms_per_frame','frame_hbm_frac')})"
done
bash scripts/gpu_r4e.sh
