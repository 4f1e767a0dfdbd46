#!/bin/bash
# C4's K = 8 band (16 200 waves, 2.3 dispatch rounds): exact pass automatic / off, 8- vs 16-row
# blocks, ranks 0 and 2, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s53}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify --config C4 --rehearse-ranks 8"
for round in 1 2; do
for spec in "0 1 8" "0 0 8" "0 1 16" "2 1 8" "2 0 8" "2 1 16"; do
  set -- $spec
  timeout -k 10 200 python bench.py --rehearse-rank $1 --exact-pass $2 --row-block $3 $B > $OUT/C4_r$1_e$2_b$3_$round.log 2>&1 || exit 1
  echo "r$round C4 k8 rank$1 exact$2 block$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/C4_r$1_e$2_b$3_$round.log)"
done; done
