#!/bin/bash
# Every rank's band of a K-way split, rehearsed on one GPU, per library (the product + the
# build/variants/*.so), slowest band last: bash scripts/bands_ab.sh TAG CFG K [STEPS]
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$1; mkdir -p $OUT
for lib in base $(ls build/variants/*.so 2>/dev/null); do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
  worst=0
  for ((r = 0; r < $3; r++)); do
    timeout -k 10 120 python bench.py --config $2 --rehearse-ranks $3 --rehearse-rank $r --steps ${4:-300} \
      --warmup 50 --cpu-seconds 0 --no-verify > $OUT/bands_${ln}_$2_k$3_r$r.log 2>&1 || exit 3
    km=$(grep -o '"kernel_ms": [0-9.]*' $OUT/bands_${ln}_$2_k$3_r$r.log | head -1 | grep -o '[0-9.]*$')
    worst=$(python3 -c "print(max($worst, ${km:-0}))")
  done
  echo "bands $ln $2 k$3 slowest $worst"
done
