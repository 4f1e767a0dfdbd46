#!/bin/bash
# Block-cyclic bands (ABI v11) in the one-GPU strong-scaling rehearsal: GPU tests of the block
# entry points, then rank 0's band with 8-row blocks (the bench default) against cyclic rows at
# K = 2 / 4 / 8, then every rank's band at K = 8 (the K-GPU frame is the slowest rank's).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s45}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_block_bands.py \
  tests/test_gpu_tiles.py tests/test_gpu_bench_multirank.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
B="--cpu-seconds 0 --steps 500 --warmup 200"
for cfg in C4 C3; do
  for K in 2 4 8; do
    for RB in 8 1; do
      timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks $K --row-block $RB $B > $OUT/${cfg}_k${K}_b${RB}.log 2>&1 || exit $?
      echo "$cfg k$K b$RB $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_k${K}_b${RB}.log | head -1) $(grep -o '"verified": [a-z]*' $OUT/${cfg}_k${K}_b${RB}.log | head -1)"
    done
  done
  for R in 1 2 3 4 5 6 7; do
    timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks 8 --rehearse-rank $R --no-verify $B > $OUT/${cfg}_k8_b8_r$R.log 2>&1 || exit $?
    echo "$cfg k8 b8 rank$R $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_k8_b8_r$R.log | head -1)"
  done
done
