#!/bin/bash
# Frames in flight (lanes) for the slowest rank's 8-row-block band at K = 8 (C3 rank 4, C4 rank 2,
# r03_s45) and the whole frame: does a deeper pipeline hide the band's slowest waves?
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s47}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for spec in "C3 8 4" "C4 8 2" "C3 1 0" "C4 1 0"; do
  set -- $spec
  for L in 4 6 8; do
    timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 --rehearse-rank $3 --lanes $L $B > $OUT/$1_k$2_r$3_l$L.log 2>&1 || exit $?
    echo "$1 k$2 rank$3 lanes$L $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_k$2_r$3_l$L.log | head -1)"
  done
done
