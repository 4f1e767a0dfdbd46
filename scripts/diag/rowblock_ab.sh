#!/bin/bash
# Block-cyclic bands (build/variants/libvrt_rb8.so: rank r renders 8-row blocks r, r+K, ...)
# against cyclic rows (product library) in the one-GPU strong-scaling rehearsal, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s44}; mkdir -p $OUT
for round in 1 2; do
for lib in base build/variants/libvrt_rb8.so; do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for ck in "C4 8" "C3 8" "C4 4" "C3 4" "C4 2"; do
    set -- $ck
    timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 --cpu-seconds 0 --no-verify --steps 500 --warmup 200 > $OUT/${ln}_$1_k$2_$round.log 2>&1 || exit $?
    echo "r$round $ln $1 k$2 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_$1_k$2_$round.log | head -1)"
  done
done; done
