#!/bin/bash
# Build a library variant for same-box A/B (MTTS_LIB): one source recompiled with extra defines,
# linked with the default build's other objects.
#   bash scripts/mkvar.sh NAME "-DPSE_APAUSE=1" [pse.hip [FILE]]   -> moss_tts_amd/lib/var/libmtts_NAME.so
# FILE (optional, absolute): compiled in place of src, e.g. an earlier revision of it for a before / after
set -eu
cd "$(dirname "$0")/../moss_tts_amd/csrc"
name=$1; defs=$2; src=${3:-pse.hip}; file=${4:-$src}
make -s -j8 >/dev/null
mkdir -p build/var ../lib/var
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-result -Wno-unused-value -ffp-contract=fast \
  -I. $defs -x hip -c $file -o build/var/${src}_$name.o
objs=$(for s in $(sed -n "s/^SRCS = //p" Makefile); do [ "$s" = "$src" ] || echo build/$s.o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/var/libmtts_$name.so $objs build/build_id.o build/var/${src}_$name.o
echo "built moss_tts_amd/lib/var/libmtts_$name.so"
