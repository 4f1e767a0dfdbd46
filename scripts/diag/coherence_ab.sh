#!/bin/bash
# Row-interleave coherence cost: the whole frame rendered as 1 part (row_step 1) against 8 and 4
# interleaved parts (row_step 8 / 4: the tile shape of a K-way cyclic band), four lanes in flight,
# so the device stays saturated and only the walks' coherence differs; then the K = 8 band.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s43}; mkdir -p $OUT
for cfg in C4 C3; do
  for P in 1 8 4; do
    timeout -k 10 200 python bench.py --config $cfg --parts $P --lanes 4 --cpu-seconds 0 --no-verify --steps 400 --warmup 100 > $OUT/${cfg}_parts$P.log 2>&1 || exit $?
    echo "$cfg parts $P $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_parts$P.log | head -1)"
  done
  timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks 8 --cpu-seconds 0 --no-verify --steps 400 --warmup 100 > $OUT/${cfg}_k8.log 2>&1 || exit $?
  echo "$cfg k8 $(grep -o '"kernel_ms": [0-9.]*' $OUT/${cfg}_k8.log | head -1)"
done
