#!/bin/bash
# Rehearsed bands with the exact pass automatic (1) vs forced (2): bench.py --rehearse-ranks K
# --exact-pass E for the given ranks. Usage: bash scripts/rehearse_exact.sh TAG CFG K "RANKS" [RUNS]
cd "${GRAFT_REPO_ROOT:-.}"; TAG=$1; CFG=$2; K=$3; RANKS=$4; R=${5:-1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do for e in 1 2; do for r in $RANKS; do
  f=$OUT/${CFG}_k${K}_r${r}_e${e}_$i.log
  timeout -k 10 120 python bench.py --config $CFG --rehearse-ranks $K --rehearse-rank $r --exact-pass $e \
    --steps 400 --warmup 100 --cpu-seconds 0 --no-verify > $f 2>&1 || exit $?
  echo "$CFG k$K r$r exact-pass $e run $i $(grep -o '"kernel_ms": [0-9.]*' $f | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $f | head -1)"
done; done; done
