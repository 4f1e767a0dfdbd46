#!/bin/bash
# GPU check of the ABI v8 frame API and the bench path, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-s05}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame_api.py tests/test_gpu_bench_path.py -x -v -s --timeout 300 --timeout-method thread > $OUT/new.log 2>&1; rc=$?
echo "== new rc=$rc"; grep -v amdgpu.ids $OUT/new.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "== all rc=$rc"; tail -5 $OUT/pytest_gpu.log
exit $rc
