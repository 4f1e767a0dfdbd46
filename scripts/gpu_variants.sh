#!/bin/bash
# A/B of build/variants/*.so against the product library through bench.py (steady state), two
# alternating rounds; then lane counts on the product library.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s11}; mkdir -p $OUT
for round in 1 2; do
for lib in base $(ls build/variants/*.so); do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for cfgsh in "C3 color" "C2 color" "C4 color" "C3 textured"; do
    set -- $cfgsh
    timeout -k 10 200 python bench.py --config $1 --shading $2 --cpu-seconds 0 --no-verify --steps 400 --warmup 100 > $OUT/${ln}_$1_$2_$round.log 2>&1 || exit $?
    echo "r$round $ln $1 $2 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_$1_$2_$round.log | head -1)"
  done
done; done
unset VRT_LIB
for L in 2 3 6 8; do
  timeout -k 10 200 python bench.py --config C3 --lanes $L --cpu-seconds 0 --no-verify > $OUT/lanes${L}_C3.log 2>&1 || exit $?
  echo "lanes $L C3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/lanes${L}_C3.log | head -1)"
done
