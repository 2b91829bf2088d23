#!/bin/bash
# Round 4 session K: gemm3 as a 4-stage 32-deep LDS-DMA ring -- prefill parity tests, B=32 / TTSD
# prefill A/B (ring depth 3, gemm3 off), MFMA-busy counters.  gpurun_out/r4k/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "prefill or gemm or packed" -m gpu -q \
    -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "prefill tests rc=$rc"; tail -2 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "512 moss_tts_amd/lib/libmtts.so" "512 moss_tts_amd/lib/var/libmtts_nst3.so" "0 moss_tts_amd/lib/libmtts.so"; do
  set -- $v
  MTTS_GEMM3_MIN=$1 MTTS_LIB=$2 timeout -k 10 300 python3 bench.py --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --no-codec \
      --no-dp-leg --no-roofline --extra-batches "" > $O/b32.json 2> $O/b32.err
  rc=$?; [ $rc -eq 0 ] || { echo "b32 $v rc=$rc"; tail -5 $O/b32.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/b32.json')); print('B=32 g3min=$1 $(basename $2)', {k: d[k] for k in ('value','prefill_ms','ms_per_decode_step')})"
  MTTS_GEMM3_MIN=$1 MTTS_LIB=$2 timeout -k 10 300 python3 bench.py --config ttsd --decode-steps 40 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-roofline > $O/ttsd.json 2> $O/ttsd.err
  rc=$?; [ $rc -eq 0 ] || { echo "ttsd $v rc=$rc"; tail -5 $O/ttsd.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/ttsd.json')); print('TTSD prefill g3min=$1 $(basename $2)', d['prefill_ms'])"
done
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d /tmp/mfma -o m \
    --output-format csv -- python3 scripts/mfma_probe.py > $O/mfma_probe.json 2> $O/mfma_probe.err
rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/mfma_probe.err; exit $rc; }
python3 scripts/mfma_probe.py --summarize /tmp/mfma > $O/pmc_mfma.json && head -30 $O/pmc_mfma.json
