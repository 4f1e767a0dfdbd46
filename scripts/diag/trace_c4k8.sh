#!/bin/bash
# Kernel durations of C4's whole frame and of its K = 8 band (rank 0), rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-r03_s59}; mkdir -p $OUT; export TMPDIR=/tmp
for K in 1 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k$K -o run --output-format csv -- python3 $ROOT/bench.py --config C4 --rehearse-ranks $K --cpu-seconds 0 --no-verify --steps 500 --warmup 200 > $OUT/k$K.log 2>&1 || exit 1
  grep -o '"kernel_ms": [0-9.]*' $OUT/k$K.log
  find $OUT/k$K -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
done
