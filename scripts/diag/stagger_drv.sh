#!/bin/bash
# The driver's shape (20 after 5) with and without staggered lane starts, C3, four processes each.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s72}; mkdir -p $OUT
for i in 1 2 3 4; do for s in "" "--stagger"; do
  tag=$([ -z "$s" ] && echo base || echo stagger)
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-verify $s > $OUT/${tag}_$i.log 2>&1 || exit 1
  echo "run$i $tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/${tag}_$i.log) $(grep -o '"kernel_ms": [0-9.]*' $OUT/${tag}_$i.log)"
done; done
