# v75: packed bounce-stack entries: certified + tile-order parity, A/B C1-C4, bench C3
cd $GRAFT_REPO_ROOT
O=gpurun_out/v75; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py tests/test_gpu_tile_order.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh v75ab C1,C2,C3,C4 || exit $?
bash scripts/gpu_bench_variants.sh v75bench C3 C3
