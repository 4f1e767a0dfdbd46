# v62: heavy-first tile order: GPU tests (tile order, certified), bench C1-C4 with and without
cd $GRAFT_REPO_ROOT
O=gpurun_out/v73; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tile_order.py tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_variants.sh v73bench C3 C3 C1
