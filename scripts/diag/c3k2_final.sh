#!/bin/bash
# C3's K = 2 band with the bench defaults (8 lanes on 8 queues since r03_s64), both ranks, both
# shapes, verified.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s65}; mkdir -p $OUT
for shape in "500 200" "20 5"; do
  set -- $shape
  for R in 0 1; do
    timeout -k 10 200 python bench.py --config C3 --rehearse-ranks 2 --rehearse-rank $R --cpu-seconds 0 --steps $1 --warmup $2 > $OUT/C3_k2_r${R}_s$1.log 2>&1 || exit 1
    echo "C3 k2 rank$R steps$1 $(grep -o '"kernel_ms": [0-9.]*' $OUT/C3_k2_r${R}_s$1.log) $(grep -o '"hw_queues": [0-9]*' $OUT/C3_k2_r${R}_s$1.log) $(grep -o '"verified": [a-z]*' $OUT/C3_k2_r${R}_s$1.log | head -1)"
  done
done
