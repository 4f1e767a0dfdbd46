#!/bin/bash
# Upper bound of hiding the deferred exact pass in strong-scaled bands: the band without its exact
# pass (diagnostic variant VRT_DIAG_SKIP_EXACT, images wrong) against the product, rank 0.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s60}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for lib in base build/variants/libvrt_skipx.so; do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for spec in "C4 8" "C4 4" "C4 2" "C3 2" "C3 4"; do
    set -- $spec
    timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 $B > $OUT/${ln}_$1_k$2.log 2>&1 || exit 1
    echo "$ln $1 k$2 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_$1_k$2.log)"
  done
done
