mkdir -p gpurun_out/r06_s36
timeout -k 10 120 python -u scripts/cert_modes_diag.py glass_cube 128 320 180 9 -36 4 45 270 4 4 > gpurun_out/r06_s36/diag.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_cert_trees.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s36/pytest_trees.log 2>&1 || exit 1
CFGS="C3:color:1 C1:color:1 C2:color:1" bash scripts/gpu_ab_head.sh r06_s36 || exit 1
timeout -k 10 600 python -u scripts/lattice_stress.py 800 > gpurun_out/r06_s36/stress.log 2>&1
