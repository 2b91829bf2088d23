#!/bin/bash
# One iteration: GPU tests ($TESTS), then the given bench commands ($BENCHES, ';'-separated
# argument lists for bench.py), each printing its key numbers.  Writes gpurun_out/iter/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/iter
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -20; exit $rc; }
fi
IFS=';' read -ra LIST <<< "${BENCHES:-}"
i=0
for b in "${LIST[@]}"; do
  i=$((i+1))
  env ${BENV:-MTTS_NONE=1} timeout -k 10 400 python3 bench.py $b > $O/b$i.json 2> $O/e$i.txt
  rc=$?; [ $rc -eq 0 ] || { echo "bench '$b' rc=$rc"; tail -5 $O/e$i.txt; exit $rc; }
  python3 - "$O/b$i.json" "$b" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["value", "ms_per_decode_step", "ms_per_frame", "prefill_ms", "p50_first_chunk_ms", "batch_sweep"]
print(sys.argv[2], {k: d[k] for k in keys if k in d}, "roof", (d.get("roofline") or {}).get("frac"))
PY
done
