mkdir -p gpurun_out/r06_s24
timeout -k 10 120 python -u scripts/cert_modes_diag.py > gpurun_out/r06_s24/diag.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_cert_trees.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s24/pytest_trees.log 2>&1 || exit 1
CFGS="C1:color:1 C3:color:1 C4:color:1 C3:color:8" bash scripts/gpu_ab_head.sh r06_s24
