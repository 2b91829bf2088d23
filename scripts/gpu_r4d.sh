#!/bin/bash
# Round 4 session D: the rest of session A (batch-4 launch variants A/B, TTSD long-context form on /
# off, B=32 gemm3 on / off), then the MossTTSLocal channel launch (session C).  gpurun_out/r4a, r4c.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest "tests/test_pse_gpu.py::test_pse_context_gate" -m gpu -q -p no:cacheprovider \
    --timeout 150 --timeout-method thread > $O/pytest_gate.log 2>&1
rc=$?; echo "gate test rc=$rc"; tail -2 $O/pytest_gate.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MTTS_LIB=moss_tts_amd/lib/var/libmtts_hcnt.so timeout -k 10 300 python -u -m pytest tests/test_b4_oracle_gpu.py -m gpu -q \
    -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest_b4_hcnt.log 2>&1
rc=$?; echo "b4 tests (hcnt lib) rc=$rc"; tail -2 $O/pytest_b4_hcnt.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in moss_tts_amd/lib/libmtts.so moss_tts_amd/lib/var/libmtts_hcnt.so moss_tts_amd/lib/var/libmtts_rc0.so moss_tts_amd/lib/var/libmtts_ns4.so; do
  MTTS_LIB=$lib timeout -k 10 300 python3 bench.py --batch 4 --steps 2 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
      --no-roofline --extra-batches "" > $O/b4.json 2> $O/b4.err
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -5 $O/b4.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('$O/b4.json')); print('$lib'.split('/')[-1], {k: d[k] for k in ('value','ms_per_decode_step','decode_step_hbm_frac')})"
done
for flag in 1 0; do
  MTTS_PSE_LONG=$flag timeout -k 10 400 python3 bench.py --config ttsd --steps 1 --warmup 0 --no-cpu-baseline \
      > $O/ttsd_long$flag.json 2> $O/ttsd_long$flag.err
  rc=$?; [ $rc -eq 0 ] || { echo "ttsd long=$flag rc=$rc"; tail -5 $O/ttsd_long$flag.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/ttsd_long$flag.json')); r=d['roofline']; print('ttsd pse_long=$flag', {k: d[k] for k in ('value','ms_per_decode_step','prefill_ms','decode_step_hbm_frac')}, r and {k: r.get(k) for k in ('frac','avg_launch_us','kernel')}, r and r.get('pse_long_launch'))"
done
for g3 in 512 0; do
  MTTS_GEMM3_MIN=$g3 timeout -k 10 300 python3 bench.py --batch 32 --steps 1 --warmup 1 --no-cpu-baseline --no-codec --no-dp-leg \
      --no-roofline --extra-batches "" > $O/b32_g3_$g3.json 2> $O/b32_g3_$g3.err
  rc=$?; [ $rc -eq 0 ] || { echo "b32 g3=$g3 rc=$rc"; tail -5 $O/b32_g3_$g3.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$O/b32_g3_$g3.json')); print('B=32 gemm3_min=$g3', {k: d[k] for k in ('value','prefill_ms','ms_per_decode_step')})"
done
bash scripts/gpu_r4c.sh
