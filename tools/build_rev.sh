#!/bin/bash
# Build the library of a git revision (its csrc + include) into abx/lib<NAME>.so for A/B timing
# against the working tree (abx/ travels to the GPU box; the in-tree library is untouched):
#   bash tools/build_rev.sh HEAD base
set -eu
cd "$(dirname "$0")/.."
REV=$1; NAME=$2; shift 2
SRC=$(mktemp -d)
git archive "$REV" vanrijn_amd/csrc include | tar -x -C "$SRC"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math"
for s in vr_render.hip vr_image.hip vr_build.hip vr_host.cpp; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -c $SRC/vanrijn_amd/csrc/$s -o $SRC/${s%.*}.o 2>/dev/null &
done
wait
mkdir -p abx
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $SRC/*.o -lz -o abx/lib$NAME.so
rm -rf "$SRC"
echo abx/lib$NAME.so
