#!/bin/bash
# Round 4 session J: A/Bs -- batch-4 attention with double-buffered chunk loads (PSE4_ADB), the long
# form's loader resuming after the slice's chunks (PSE_LONG_RESUME); parity tests on each variant.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
VA=moss_tts_amd/lib/var/libmtts_adb1.so
VL=moss_tts_amd/lib/var/libmtts_lres1.so
MTTS_LIB=$VA timeout -k 10 300 python -u -m pytest tests/test_b4_oracle_gpu.py -m gpu -q -p no:cacheprovider \
    --timeout 250 --timeout-method thread > $O/pytest_adb.log 2>&1
rc=$?; echo "b4 tests ($VA) rc=$rc"; tail -2 $O/pytest_adb.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MTTS_LIB=$VL timeout -k 10 300 python -u -m pytest tests/test_ttsd_shape_gpu.py "tests/test_pse_gpu.py::test_pse_context_gate" \
    -m gpu -q -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest_lres.log 2>&1
rc=$?; echo "ttsd tests ($VL) rc=$rc"; tail -2 $O/pytest_lres.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in moss_tts_amd/lib/libmtts.so $VA; do
    MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --batch 4 --steps 2 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
        --no-roofline --extra-batches "" > $O/b4.json 2> $O/b4.err
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b4.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/b4.json')); print('B=4', '$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step')})"
  done
done
for lib in moss_tts_amd/lib/libmtts.so $VL; do
  MTTS_LIB=$lib timeout -k 10 400 python3 bench.py --config ttsd --steps 1 --warmup 0 --no-cpu-baseline --no-roofline \
      > $O/ttsd.json 2> $O/ttsd.err
  rc=$?; [ $rc -eq 0 ] || { echo "ttsd $lib rc=$rc"; tail -5 $O/ttsd.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/ttsd.json')); print('TTSD', '$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')})"
done
