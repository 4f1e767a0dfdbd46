#!/bin/bash
# Lane-level vs wave-level step counts per config from the diagnostic builds (TIE3 slot):
# diags = sampled lane-steps, diagw1 = wave-level steps, diagw2 = wave-level sampled branches.
set -e
out=$1; mkdir -p "$out"
for v in diags diagw1 diagw2; do
  VRT_LIB=build/variants/libvrt_$v.so timeout -k 10 200 python scripts/diag_counts.py --configs C1,C2,C3,C4 \
    2>&1 | grep -v amdgpu.ids > "$out/$v.log"
done
