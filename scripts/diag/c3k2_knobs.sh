#!/bin/bash
# C3's K = 2 band (16 200 waves): deferred / in-lane exact path x 4 lanes on 4 queues / 8 on 8,
# both ranks.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s62}; mkdir -p $OUT
B="--config C3 --rehearse-ranks 2 --cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for R in 0 1; do for spec in "1 4 4" "0 4 4" "1 8 8" "0 8 8" "0 6 6"; do
  set -- $spec
  timeout -k 10 200 python bench.py --rehearse-rank $R --exact-pass $1 --queues $2 --lanes $3 $B > $OUT/r${R}_e$1_q$2_l$3.log 2>&1 || exit 1
  echo "C3 k2 rank$R exact$1 q$2 lanes$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/r${R}_e$1_q$2_l$3.log)"
done; done
