#!/bin/bash
# 8 lanes on 8 hardware queues against 4 on 4 for the deferred-pass bands (16-row blocks), rank 0,
# two rounds: C4 at K = 2 / 4 / 8, C2 at K = 2 / 4, textured C3 at K = 2.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s63}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for round in 1 2; do
for spec in "C4 color 8" "C4 color 4" "C4 color 2" "C2 color 2" "C2 color 4" "C3 textured 2"; do
  set -- $spec
  for q in 4 8; do
    timeout -k 10 200 python bench.py --config $1 --shading $2 --rehearse-ranks $3 --queues $q --lanes $q $B > $OUT/$1_$2_k$3_q${q}_$round.log 2>&1 || exit 1
    echo "r$round $1 $2 k$3 q$q lanes$q $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_$2_k$3_q${q}_$round.log)"
  done
done; done
