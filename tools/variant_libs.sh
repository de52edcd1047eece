#!/bin/bash
# Build several A/B variants of the library in parallel into abx/lib<name>.so (travels to the GPU box; git-ignored): the other three
# translation units are compiled once; each variant recompiles vr_render.hip with its own flags.
#   bash tools/variant_libs.sh base "" split "-DVR_NODE_SPLIT_LOAD" ...
set -eu
cd "$(dirname "$0")/.."
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math"
COMMON=$(mktemp -d)
mkdir -p abx
for s in vr_image.hip vr_build.hip vr_host.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -c vanrijn_amd/csrc/$s -o $COMMON/${s%.*}.o &
done
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc $FLAGS $flags -c vanrijn_amd/csrc/vr_render.hip -o $COMMON/render_$name.o 2>/dev/null ) &
  NAMES="${NAMES:-} $name"
done
wait
for name in $NAMES; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $COMMON/render_$name.o $COMMON/vr_image.o \
      $COMMON/vr_build.o $COMMON/vr_host.o -lz -o abx/lib$name.so
  echo abx/lib$name.so
done
rm -rf "$COMMON"
