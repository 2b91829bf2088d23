#!/bin/bash
# A/B of the publish-only threshold (MTTS_ATTN_PO_MAX) at long contexts (TTSD shape) and the
# default clone bench; GPU tests first.  Writes gpurun_out/po/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/po
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for tt in ${TEXT_TOKENS:-2000 8000}; do
  for po in ${POS:-256 2 4 8}; do
    MTTS_ATTN_PO_MAX=$po timeout -k 10 300 python3 bench.py --config ttsd --text-tokens $tt --decode-steps ${DSTEPS:-200} \
        --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-codec > $O/b.json 2> $O/e.txt
    rc=$?; [ $rc -eq 0 ] || { echo "po=$po tt=$tt rc=$rc"; tail -5 $O/e.txt; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/b.json'));print('text_tokens=$tt po_max=$po ms/step', d['ms_per_decode_step'])"
  done
done
