#!/bin/bash
# 8 lanes on 8 queues against 4 on 4: textured C4 at K = 8, C1 at K = 2, textured C3 at K = 1.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s64}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for spec in "C4 textured 8" "C1 color 2" "C3 textured 1"; do
  set -- $spec
  for q in 4 8; do
    timeout -k 10 200 python bench.py --config $1 --shading $2 --rehearse-ranks $3 --queues $q --lanes $q $B > $OUT/$1_$2_k$3_q$q.log 2>&1 || exit 1
    echo "$1 $2 k$3 q$q lanes$q $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_$2_k$3_q$q.log)"
  done
done
