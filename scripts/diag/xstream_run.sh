#!/bin/bash
# GPU tests of the deferred pass (incl. paired exact streams) and block bands, then the A/B.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s61}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_exact_pass.py tests/test_gpu_block_bands.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/xstream_ab.sh ${1:-r03_s61}
