cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v35
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v35/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/v35/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab.py --rounds 8 --configs C1,C2,C3,C4 > gpurun_out/v35/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/v35/ab.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/v35/bench.log 2>&1; tail -1 gpurun_out/v35/bench.log
