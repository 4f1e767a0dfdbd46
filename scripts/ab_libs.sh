#!/bin/bash
# Interleaved A/B of whole libraries through scripts/streams_exp.py (the bench's 2-stream frame
# loop): ab_libs.sh OUTDIR CONFIGS LIB1 LIB2 ... ; each library runs twice, alternating.
set -e
out=$1; cfgs=$2; shift 2
mkdir -p "$out"
for pass in 1 2; do
  for lib in "$@"; do
    VRT_LIB=$lib GPU_MAX_HW_QUEUES=16 timeout -k 10 150 \
      python scripts/streams_exp.py --configs "$cfgs" --parts 2 --frames 300 --warmup 200 \
      2>&1 | grep -v amdgpu.ids >> "$out/exp.log"
  done
done
