#!/bin/bash
# Exact-pass grid = certified waves / D: D = 8 (product) against 16 and 32 (variants), colour-only
# frames (few deferred pixels: most exact-pass waves find no batch) and textured C3, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s58}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for round in 1 2; do
for lib in base build/variants/libvrt_gd16.so build/variants/libvrt_gd32.so; do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for spec in "C3 color 1" "C4 color 1" "C4 color 8" "C2 color 1" "C3 textured 1"; do
    set -- $spec
    timeout -k 10 200 python bench.py --config $1 --shading $2 --rehearse-ranks $3 $B > $OUT/${ln}_$1_$2_k$3_$round.log 2>&1 || exit 1
    echo "r$round $ln $1 $2 k$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_$1_$2_k$3_$round.log)"
  done
done; done
