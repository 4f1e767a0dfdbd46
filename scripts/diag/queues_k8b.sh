#!/bin/bash
# C3 at K = 8: the slow ranks of r03_s51 (1, 2, 4) and rank 0 with 8 / 9 / 12 hardware queues and
# 7 / 8 lanes (is a lane sharing a queue behind the bimodal band times?).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s52}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify --rehearse-ranks 8"
for spec in "1 8 8" "1 9 8" "1 8 7" "1 12 8" "2 8 8" "2 9 8" "2 8 7" "4 8 8" "4 9 8" "4 8 7" "0 9 8" "0 8 7"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config C3 --rehearse-rank $1 --queues $2 --lanes $3 $B > $OUT/C3_r$1_q$2_l$3.log 2>&1 || exit 1
  echo "C3 k8 rank$1 q$2 lanes$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/C3_r$1_q$2_l$3.log)"
done
