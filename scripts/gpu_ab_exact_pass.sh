#!/bin/bash
# r03: deferred exact pass A/B. Tests first, then bench per config with the pass on / off.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s6}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_pass.py tests/test_gpu_certified.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
for cfg in ${CFGS:-C3 C2 C1 C4}; do for ep in 1 0 1 0; do
  timeout -k 10 200 python bench.py --config $cfg --exact-pass $ep --cpu-seconds 0 ${EXTRA} > $OUT/b_${cfg}_ep${ep}.log 2>&1 || exit $?
  echo "$cfg ep=$ep $(grep -o '"kernel_ms": [0-9.]*\|"verified": [a-z]*' $OUT/b_${cfg}_ep${ep}.log | head -2 | tr '\n' ' ')"
done; done
