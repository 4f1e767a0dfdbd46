#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s10}; mkdir -p $OUT
for sh in color textured; do for cf in 0 1; do for ep in 1 0; do
  timeout -k 10 200 python bench.py --config C1 --shading $sh --certified $cf --exact-pass $ep --cpu-seconds 0 > $OUT/c1_${sh}_cf${cf}_ep${ep}.log 2>&1 || exit $?
  echo "C1 $sh certified=$cf ep=$ep $(grep -o '"kernel_ms": [0-9.]*\|"verified": [a-z]*' $OUT/c1_${sh}_cf${cf}_ep${ep}.log | head -2 | tr '\n' ' ')"
done; done; done
