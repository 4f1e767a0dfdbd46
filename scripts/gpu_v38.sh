cd $GRAFT_REPO_ROOT
O=gpurun_out/v38; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cert.log 2>&1; rc=$?; tail -15 $O/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab.py --rounds 8 --configs C1,C2,C3,C4 > $O/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.log | grep -v '^{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; tail -1 $O/bench.log
