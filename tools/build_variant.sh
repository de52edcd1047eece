#!/bin/bash
# Build an A/B variant of the library with extra compile flags into ab/lib<name>.so
# (the in-tree library is untouched):  bash tools/build_variant.sh NAME -DVR_PEND=12 ...
set -eu
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=$(mktemp -d)
FLAGS="--offload-arch=gfx950 ${OPT:--O3} -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Xarch_device -mllvm=-amdgpu-use-amdgpu-trackers"
pids=()
for s in vr_render.hip vr_image.hip vr_build.hip vr_host.cpp; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -c vanrijn_amd/csrc/$s -o $OUT/${s%.*}.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done  # set -e: a failed compile stops the link
D=${OUTDIR:-ab}
mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/*.o -lz -o $D/lib$NAME.so
rm -rf "$OUT"
echo $D/lib$NAME.so
