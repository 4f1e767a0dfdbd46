#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=$(pwd)/gpurun_out/${1:-diag}; mkdir -p $OUT; export TMPDIR=/tmp
A="build/bin/vrt_headless --scene refraction --n 128 --size 1920x1080 --bounces 4 4 --frames 300 --warmup 100 --quiet"
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/pipe -o run --output-format csv -- $A --pipelined > $OUT/pipe.log 2>&1; echo "pipe rc=$?"; grep pipelined $OUT/pipe.log
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/sync -o run --output-format csv -- $A > $OUT/sync.log 2>&1; echo "sync rc=$?"; grep timed $OUT/sync.log
