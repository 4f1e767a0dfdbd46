#!/bin/bash
# C3 K = 8 band (8 lanes on 8 queues): is the per-process bimodality (0.0073 vs 0.0105 ms) the
# heavy-first tile order? Rank 4, four processes each with the order on and off.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s57}; mkdir -p $OUT
B="--config C3 --rehearse-ranks 8 --rehearse-rank 4 --cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for i in 1 2 3 4; do for t in 1 0; do
  timeout -k 10 200 python bench.py --tile-order $t $B > $OUT/r4_t${t}_$i.log 2>&1 || exit 1
  echo "run$i tile_order$t $(grep -o '"kernel_ms": [0-9.]*' $OUT/r4_t${t}_$i.log)"
done; done
