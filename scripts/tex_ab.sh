#!/bin/bash
# Textured and colour-only frame rates per library (the product + build/variants/*.so), ROUNDS
# alternating: bash scripts/tex_ab.sh TAG [ROUNDS]
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p $OUT
for ((i = 1; i <= ${2:-2}; i++)); do
  for lib in base $(ls build/variants/*.so 2>/dev/null); do
    ln=$(basename $lib .so)
    if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
    for run in "C4 textured" "C3 textured" "C3 color" "C4 color"; do
      read cfg sh <<< "$run"
      lg=$OUT/ab_${ln}_${cfg}_${sh}_$i.log
      timeout -k 10 200 python bench.py --config $cfg --shading $sh --steps 300 --warmup 50 --cpu-seconds 0 --no-verify > $lg 2>&1 || exit 3
      echo "ab $ln $cfg $sh $i $(grep -o '"ms_per_step": [0-9.]*' $lg) $(grep -o '"frame_latency_ms": [0-9.]*' $lg | head -1)"
    done
  done
done
