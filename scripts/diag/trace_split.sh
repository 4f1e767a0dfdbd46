#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=$(pwd)/gpurun_out/${1:-ts}; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in C3 C2; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 50 --warmup 20 --cpu-seconds 0 --no-verify > $OUT/$cfg.log 2>&1; echo "$cfg rc=$?"
grep -E "cert_pass|exact_pass" $OUT/$cfg/run_kernel_stats.csv | cut -d, -f1-6
done
