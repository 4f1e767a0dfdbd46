# v50: certified shadows from exact hit points on the certified instance's exact path
cd $GRAFT_REPO_ROOT
O=gpurun_out/v53; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cert.log 2>&1; rc=$?; tail -3 $O/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh v53ab C1,C3
