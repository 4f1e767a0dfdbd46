#!/bin/bash
# NOTE: needs profiles/r03_s61/xstream.patch (the paired exact-stream experiment, reverted) for --exact-stream
# Deferred exact passes on paired streams (--exact-stream 1: 4 lane streams x 2 buffers + 4 exact
# streams, 8 hardware queues) against the default, verified frames, rank 0.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s61}; mkdir -p $OUT
B="--cpu-seconds 0 --steps 500 --warmup 200"
for round in 1 2; do
for spec in "C4 color 8" "C3 color 2" "C4 color 4" "C4 color 2" "C4 color 1" "C3 color 1" "C3 textured 1" "C3 textured 4"; do
  set -- $spec
  for x in 0 1; do
    timeout -k 10 200 python bench.py --config $1 --shading $2 --rehearse-ranks $3 --exact-stream $x $B > $OUT/$1_$2_k$3_x${x}_$round.log 2>&1 || { tail -5 $OUT/$1_$2_k$3_x${x}_$round.log; exit 1; }
    echo "r$round $1 $2 k$3 xstream$x $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_$2_k$3_x${x}_$round.log) $(grep -o '"verified": [a-z]*' $OUT/$1_$2_k$3_x${x}_$round.log | head -1)"
  done
done; done
