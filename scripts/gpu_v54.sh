# v54: full GPU suite + A/B of exact-path certification (mode 1 shadows, mode 2 shadows + secondaries)
cd $GRAFT_REPO_ROOT
O=gpurun_out/v58; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh v58ab C1,C2,C3,C4
