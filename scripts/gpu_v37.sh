cd $GRAFT_REPO_ROOT
O=gpurun_out/v37; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ab.py --rounds 8 --configs C1,C2,C3,C4 > $O/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.log | head -24; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; tail -1 $O/bench.log
