#!/bin/bash
# The driver's shape (20 frames after 5): 4 lanes on 4 queues against 8 on 8 for C3's bands at
# K = 2 and K = 8 (rank 0) and the whole frame, three processes each.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s66}; mkdir -p $OUT
B="--config C3 --cpu-seconds 0 --steps 20 --warmup 5 --no-verify"
for i in 1 2 3; do for K in 2 8 1; do for q in 4 8; do
  timeout -k 10 200 python bench.py --rehearse-ranks $K --queues $q --lanes $q $B > $OUT/k${K}_q${q}_$i.log 2>&1 || exit 1
  echo "run$i C3 k$K q$q $(grep -o '"kernel_ms": [0-9.]*' $OUT/k${K}_q${q}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/k${K}_q${q}_$i.log)"
done; done; done
