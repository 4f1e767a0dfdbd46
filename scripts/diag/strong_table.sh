#!/bin/bash
# The strong-scaling rehearsal table with bench.py's defaults (8-row blocks for split frames; 8 lanes
# on 8 hardware queues for bands below one dispatch round): every rank's band at K = 2 / 4 / 8 for
# C3 and C4, in the 500-after-200 shape and the driver's 20-after-5 shape; the K-GPU frame is the
# slowest rank's.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s51}; mkdir -p $OUT
for cfg in C3 C4; do
  for shape in "500 200" "20 5"; do
    set -- $shape
    timeout -k 10 200 python bench.py --config $cfg --cpu-seconds 0 --steps $1 --warmup $2 --no-verify > $OUT/${cfg}_k1_s$1.log 2>&1 || exit 1
    echo "$cfg k1 steps$1 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_k1_s$1.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/${cfg}_k1_s$1.log)"
    for K in 2 4 8; do
      for ((R = 0; R < K; R++)); do
        timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks $K --rehearse-rank $R --cpu-seconds 0 --steps $1 --warmup $2 --no-verify > $OUT/${cfg}_k${K}_r${R}_s$1.log 2>&1 || exit 1
        echo "$cfg k$K rank$R steps$1 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_k${K}_r${R}_s$1.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/${cfg}_k${K}_r${R}_s$1.log) $(grep -o '"hw_queues": [0-9]*' $OUT/${cfg}_k${K}_r${R}_s$1.log)"
      done
    done
  done
done
