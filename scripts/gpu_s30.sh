mkdir -p gpurun_out/r06_s34
CFGS="C3:color:1 C1:color:1 C2:color:1 C4:color:1" bash scripts/gpu_ab_head.sh r06_s34 || exit 1
timeout -k 10 600 python -u scripts/lattice_stress.py 600 > gpurun_out/r06_s34/stress.log 2>&1
