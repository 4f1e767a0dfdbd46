#!/bin/bash
# r03: textured certified pixels + exact pass: parity tests, then textured / colour benches.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s9}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact_pass.py tests/test_gpu_parity.py tests/test_gpu_certified.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-C3 C2 C1 C4}; do for ep in 1 0; do
  timeout -k 10 200 python bench.py --config $cfg --shading textured --exact-pass $ep --cpu-seconds 0 > $OUT/tex_${cfg}_ep${ep}.log 2>&1 || exit $?
  echo "tex $cfg ep=$ep $(grep -o '"kernel_ms": [0-9.]*\|"verified": [a-z]*' $OUT/tex_${cfg}_ep${ep}.log | head -2 | tr '\n' ' ')"
done; done
