#!/bin/bash
# AddressSanitizer run of libmtts's host code through the C-ABI driver (tests/native/asan_driver,
# built beforehand here: make -C tests/native).  Leaks inside the ROCm runtime are suppressed
# (tests/native/lsan.supp); anything in engine.cpp / local.cpp / codec.cpp is reported.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/asan
export ASAN_OPTIONS=detect_leaks=1:protect_shadow_gap=0:halt_on_error=1:verify_asan_link_order=0
export LSAN_OPTIONS=suppressions=$PWD/tests/native/lsan.supp:print_suppressions=1
timeout -k 10 300 tests/native/asan_driver > gpurun_out/asan/asan.log 2>&1
rc=$?; echo "asan driver rc=$rc"; tail -40 gpurun_out/asan/asan.log; exit $rc
