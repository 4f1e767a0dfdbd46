#!/bin/bash
# Repeatability / pipeline-depth probe of rehearsed bands: bench.py --rehearse-ranks K for the given
# ranks and (lanes, queues) shapes, R runs each. Usage: bash scripts/rehearse_repeat.sh TAG CFG K "RANKS" "L:Q ..." R
cd "${GRAFT_REPO_ROOT:-.}"; TAG=$1; CFG=$2; K=$3; RANKS=$4; SHAPES=$5; R=${6:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do for sh in $SHAPES; do for r in $RANKS; do
  IFS=: read l q <<< "$sh"
  f=$OUT/${CFG}_k${K}_r${r}_l${l}q${q}_$i.log
  timeout -k 10 120 python bench.py --config $CFG --rehearse-ranks $K --rehearse-rank $r --lanes $l --queues $q \
    --steps 400 --warmup 100 --cpu-seconds 0 --no-verify > $f 2>&1 || exit $?
  echo "$CFG k$K r$r lanes $l queues $q run $i $(grep -o '"kernel_ms": [0-9.]*' $f | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $f | head -1)"
done; done; done
