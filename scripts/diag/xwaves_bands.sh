#!/bin/bash
# Exact-pass occupancy (VRT_EXACT_WAVES 7 product, 5 and 4: fewer waves, more VGPRs, fewer spills)
# on the exact-pass-bound bands (C4 K = 8, C3 K = 2, textured C4 K = 8) and whole frames, rank 0.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s67}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for lib in base build/variants/libvrt_xw5.so build/variants/libvrt_xw4.so; do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for spec in "C4 color 8" "C3 color 2" "C4 textured 8" "C4 color 1" "C3 color 1"; do
    set -- $spec
    timeout -k 10 200 python bench.py --config $1 --shading $2 --rehearse-ranks $3 $B > $OUT/${ln}_$1_$2_k$3.log 2>&1 || exit 1
    echo "$ln $1 $2 k$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_$1_$2_k$3.log)"
  done
done
