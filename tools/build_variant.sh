#!/bin/bash
# Build a measurement variant of libvcg_hip.so: one source file recompiled with extra flags, linked with the main
# build's other objects (run `make` in csrc first). usage: tools/build_variant.sh <source.hip> <out.so> <flags...>
# e.g. tools/build_variant.sh igemm_wide.hip video-chapter-generation_amd/vcg_hip/libvcg_wide_stamps.so -DVCG_WIDE_STAMPS
set -e
SRC=$1; OUT=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/video-chapter-generation_amd/csrc
OBJ=$ROOT/video-chapter-generation_amd/build/obj
TMP=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -w "$@" -c "$CSRC/$SRC" -o "$TMP/v.o"
OTHERS=$(for f in "$CSRC"/*.hip; do b=$(basename "${f%.hip}"); [ "$b" != "${SRC%.hip}" ] && echo "$OBJ/$b.o"; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" "$TMP/v.o" $OTHERS -ldl
rm -rf "$TMP"
echo "built $OUT"
