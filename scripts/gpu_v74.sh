# v74: certified-walk parity incl. glass slabs (continuations)
cd $GRAFT_REPO_ROOT
O=gpurun_out/v74; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cert.log 2>&1; rc=$?; tail -4 $O/pytest_cert.log; exit $rc
