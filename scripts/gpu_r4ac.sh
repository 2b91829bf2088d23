#!/bin/bash
# Round 4 session AC: the ASan driver alone (timed, verbose), then the GPU tests after it in collection
# order, verbose so that progress shows.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4ac
mkdir -p $O
start=$(date +%s)
timeout -k 10 400 python -u -m pytest -x -v --timeout 350 --timeout-method thread tests/test_native_asan_gpu.py -p no:cacheprovider > $O/asan.txt 2>&1
rc=$?; echo "asan rc=$rc in $(( $(date +%s) - start )) s"; tail -3 $O/asan.txt; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_pse_gpu.py tests/test_pse_oracle_gpu.py tests/test_reference_ids_gpu.py tests/test_sampling_gpu.py tests/test_splitk2_gpu.py tests/test_ttsd_shape_gpu.py -p no:cacheprovider > $O/rest.txt 2>&1
rc=$?; echo "rest rc=$rc"; tail -3 $O/rest.txt
