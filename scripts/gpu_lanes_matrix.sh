#!/bin/bash
# Lanes x exact pass x band size (one-GPU rehearsal of a K-way split) in both run shapes.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s19}; mkdir -p $OUT
for cfg in ${CFGS:-C3}; do for k in ${KS:-1 4 8}; do for L in ${LANES:-2 4 8}; do for ep in 1 0; do
  for shape in "--steps 20 --warmup 5" "--steps 500 --warmup 200"; do
    tag=${cfg}_k${k}_L${L}_ep${ep}_$(echo $shape | cut -d' ' -f2)
    timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks $k --lanes $L --exact-pass $ep $shape --cpu-seconds 0 --no-verify > $OUT/$tag.log 2>&1 || exit $?
    echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $OUT/$tag.log | head -1)"
  done
done; done; done; done
