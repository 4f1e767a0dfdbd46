#!/bin/bash
# Build the product library of git revision REV as an A/B variant: build/variants/libvrt_NAME.so
# Usage: bash scripts/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2; ROOT=$(cd "$(dirname "$0")/.." && pwd); D=$ROOT/build/rev/$NAME
rm -rf "$D"; mkdir -p "$D/include" "$D/csrc" "$ROOT/build/variants"
git -C "$ROOT" show "$REV:include/vrt.h" > "$D/include/vrt.h"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" voxelraytracer_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$D/csrc/$(basename $f)"
done
SRCS=$(ls $D/csrc/*.hip $D/csrc/*.cpp)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I$D/include -I$D/csrc -DVRT_DIAGNOSTIC_BUILD \
  -shared -o $ROOT/build/variants/libvrt_$NAME.so $SRCS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $NAME from $REV"
