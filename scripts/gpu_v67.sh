# v67: tile order only with glass in the volume: GPU suite, bench C1-C4 with and without
cd $GRAFT_REPO_ROOT
O=gpurun_out/v67; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_variants.sh v67bench C3 C1 C2 C4
