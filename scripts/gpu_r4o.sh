#!/bin/bash
# Round 4 session O: shared chunk step (pse_chunk.h) in all three persistent attention bodies.
# PSE / batch-4 parity tests, then B=4, TTSD and B=1 decode step times against the previous pse4.hip
# (moss_tts_amd/lib/var/libmtts_p4head.so), twice each.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_pse_gpu.py tests/test_ttsd_shape_gpu.py tests/test_pse_oracle_gpu.py tests/test_b4_oracle_gpu.py > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
for lib in moss_tts_amd/lib/libmtts.so moss_tts_amd/lib/var/libmtts_p4head.so; do
  MTTS_LIB=$lib timeout -k 10 300 python bench.py --batch 4 --steps 3 --no-cpu-baseline --no-codec --no-roofline --no-dp-leg --extra-batches "" > $O/b.json 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$lib B=4', d['value'], d['ms_per_decode_step'])"
done
done
lib=moss_tts_amd/lib/libmtts.so
MTTS_LIB=$lib timeout -k 10 300 python bench.py --config ttsd --steps 3 --no-cpu-baseline --no-codec --no-roofline > $O/t.json 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/t.json'));print('$lib ttsd', d['value'], d['ms_per_decode_step'])"
MTTS_LIB=$lib timeout -k 10 300 python bench.py --batch 1 --steps 3 --no-cpu-baseline --no-codec --no-roofline --no-dp-leg --extra-batches "" > $O/b.json 2> $O/e.txt || { tail -3 $O/e.txt; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print('$lib B=1', d['value'], d['ms_per_decode_step'])"
