#!/bin/bash
# The exact pass's 4-wave instance for colour-only bands of < 4 rounds (a.exact_fat): GPU tests,
# then the affected bands and unaffected whole frames, two rounds (before: C4 k8 0.0229, C3 k2
# 0.0275, C2 k2 0.0338, C4 0.1389, C3 0.0387 ms; r03_s63, r03_s67).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s68}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_exact_pass.py tests/test_gpu_block_bands.py tests/test_gpu_bench_path.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="--cpu-seconds 0 --steps 500 --warmup 200"
for round in 1 2; do
for spec in "C4 8" "C3 2" "C2 2" "C4 1" "C3 1"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --rehearse-ranks $2 $B > $OUT/$1_k$2_$round.log 2>&1 || exit 1
  echo "r$round $1 k$2 $(grep -o '"kernel_ms": [0-9.]*' $OUT/$1_k$2_$round.log) $(grep -o '"verified": [a-z]*' $OUT/$1_k$2_$round.log | head -1)"
done; done
