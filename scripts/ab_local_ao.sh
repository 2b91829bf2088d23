#!/bin/bash
# MossTTSLocal fused depth attention + o_proj (local_ao.hip): the B = 8 parity tests on both forms,
# then a same-box A/B of the frame (MTTS_LOCAL_AO=0 / 1).  Writes gpurun_out/ab_local_ao/.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_local_ao
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_local_b8_gpu.py tests/test_local_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for ao in 0 1; do
    MTTS_LOCAL_AO=$ao timeout -k 10 300 python bench.py --config local --steps 2 --warmup 1 --no-cpu-baseline \
        > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/l.json'));print('local_ao $ao', d['ms_per_frame'], 'ms/frame', d['value'])" | tee -a $O/summary.txt
  done
done
