#!/bin/bash
# Every rank's band (rank-to-rank spread) for cyclic rows and 8-row blocks where r03_s45 timed only
# rank 0: C3 at K = 2 / 4 / 8 and C4 at K = 8.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s46}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200 --no-verify"
for spec in "C3 2 8" "C3 2 1" "C3 4 8" "C3 4 1" "C3 8 1" "C4 8 1"; do
  set -- $spec
  for ((R = 0; R < $2; R++)); do
    timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 --rehearse-rank $R --row-block $3 $B > $OUT/$1_k$2_b$3_r$R.log 2>&1 || exit $?
    echo "$1 k$2 b$3 rank$R $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_k$2_b$3_r$R.log | head -1)"
  done
done
