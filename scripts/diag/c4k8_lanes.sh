#!/bin/bash
# C4's K = 8 band (rank 0) with 4 / 5 / 6 lanes, each on its own hardware queue, in both shapes.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s70}; mkdir -p $OUT
for shape in "500 200" "20 5" "20 5"; do
  set -- $shape
  for q in 4 5 6; do
    timeout -k 10 200 python bench.py --config C4 --rehearse-ranks 8 --queues $q --lanes $q --cpu-seconds 0 --no-verify --steps $1 --warmup $2 > $OUT/q${q}_s$1_$RANDOM.log 2>&1 || exit 1
    echo "C4 k8 q$q lanes$q steps$1 $(grep -ho '"kernel_ms": [0-9.]*' $(ls -t $OUT/q${q}_s$1_*.log | head -1)) $(grep -ho '"ms_per_step": [0-9.]*' $(ls -t $OUT/q${q}_s$1_*.log | head -1))"
  done
done
