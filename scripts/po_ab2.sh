#!/bin/bash
# full GPU tests, then the publish-only threshold A/B at long contexts and the B=1/B=32 benches
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/po
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
for tt in ${TEXT_TOKENS:-2000 8000}; do
  for po in ${POS:-256 1 2 4}; do
    MTTS_ATTN_PO_MAX=$po timeout -k 10 300 python3 bench.py --config ttsd --text-tokens $tt --decode-steps ${DSTEPS:-200} \
        --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-codec > $O/b.json 2> $O/e.txt
    rc=$?; [ $rc -eq 0 ] || { echo "po=$po tt=$tt rc=$rc"; tail -5 $O/e.txt; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/b.json'));print('text_tokens=$tt po_max=$po ms/step', d['ms_per_decode_step'])"
  done
done
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-codec --extra-batches 4,32 > $O/clone.json 2> $O/e.txt
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/e.txt; exit $rc; }
python3 -c "import json;d=json.load(open('$O/clone.json'));print('clone B=1', d['value'], d['ms_per_decode_step'], d['batch_sweep'])"
