#!/bin/bash
# Synchronous-frame latency (bench.py's latency.sync_frame_kernel_ms: vrt_render_frame, device
# timestamps) per library x config, ROUNDS alternating: bash scripts/sync_ab.sh TAG [ROUNDS] [CFGS]
# libraries: the product (base) and build/variants/*.so
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p $OUT
for ((i = 1; i <= ${2:-2}; i++)); do
  for lib in base $(ls build/variants/*.so 2>/dev/null); do
    ln=$(basename $lib .so)
    if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
    for cfg in ${3:-C1 C2 C3 C4}; do
      timeout -k 10 120 python bench.py --config $cfg --steps 50 --warmup 10 --cpu-seconds 0 --no-verify > $OUT/sync_${ln}_${cfg}_$i.log 2>&1 || exit 3
      echo "sync $ln $cfg $i $(grep -o '"sync_frame_kernel_ms": [0-9.]*' $OUT/sync_${ln}_${cfg}_$i.log) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/sync_${ln}_${cfg}_$i.log | head -1)"
    done
  done
done
