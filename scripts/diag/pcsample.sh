#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=$(pwd)/gpurun_out/${1:-pcs}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/pc -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-verify --parts 1 > $OUT/pc.log 2>&1; echo "rc=$?"; tail -5 $OUT/pc.log; ls -la $OUT/pc 2>/dev/null | head
