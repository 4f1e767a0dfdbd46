#!/bin/bash
# A/B of the working tree's library against build/variants/*.so through bench.py (steady state,
# two alternating rounds, also the one-GPU rehearsal of rank 0's band at K = 8), after the exact-pass
# parity tests. CFGS / EXTRA override the configs / bench flags.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_pass.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
for lib in base $(ls build/variants/*.so); do
  ln=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$PWD/$lib; fi
  for cfgsh in ${CFGS:-"C3:color:1" "C2:color:1" "C4:color:1" "C3:textured:1" "C3:color:8" "C4:color:8"}; do
    IFS=: read cfg sh k <<< "$cfgsh"
    timeout -k 10 200 python bench.py --config $cfg --shading $sh --rehearse-ranks $k --cpu-seconds 0 --no-verify --steps 400 --warmup 100 $EXTRA > $OUT/${ln}_${cfg}_${sh}_k${k}_$round.log 2>&1 || exit $?
    echo "r$round $ln $cfg $sh k$k $(grep -o '"kernel_ms": [0-9.]*' $OUT/${ln}_${cfg}_${sh}_k${k}_$round.log | head -1)"
  done
done; done
