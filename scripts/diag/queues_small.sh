#!/bin/bash
# 8 hardware queues x 8 lanes against 4 x 4 for bands below / around one dispatch round of waves:
# every rank of C3 at K = 8 and K = 4, rank 0 of C1 / C2 at K = 8 (r03_s49: C3 k8 rank 4 0.0138 ->
# 0.0105 ms, C4 k8 rank 2 0.0236 -> 0.0275).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s50}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
run() {  # cfg K rank queues lanes
  GPU_MAX_HW_QUEUES=$4 timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 --rehearse-rank $3 --lanes $5 $B > $OUT/$1_k$2_r$3_q$4_l$5.log 2>&1 || exit 1
  echo "$1 k$2 rank$3 q$4 lanes$5 $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_k$2_r$3_q$4_l$5.log)"
}
for R in 0 1 2 3 4 5 6 7; do run C3 8 $R 8 8; done
for R in 0 1 2 3; do run C3 4 $R 8 8; run C3 4 $R 4 4; done
for c in C1 C2; do run $c 8 0 4 4; run $c 8 0 8 8; done
