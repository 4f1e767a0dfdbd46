#!/bin/bash
# Row-block size 8 / 16 / 32 for rank 0's band (rank 0 always holds the most blocks), C3 and C4 at
# K = 2 / 4 / 8.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s54}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for spec in "C4 8 32" "C4 8 16" "C4 8 8" "C4 4 16" "C4 4 8" "C4 2 16" "C4 2 8" "C3 2 16" "C3 2 8" "C3 4 16" "C3 4 8" "C3 8 16" "C3 8 8"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 --row-block $3 $B > $OUT/$1_k$2_b$3.log 2>&1 || exit 1
  echo "$1 k$2 block$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_k$2_b$3.log)"
done
