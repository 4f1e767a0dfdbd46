#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-diag}; mkdir -p $OUT
A="build/bin/vrt_headless --scene refraction --n 128 --size 1920x1080 --bounces 4 4 --frames 400 --warmup 200"
timeout -k 10 120 $A > $OUT/app_default.log 2>&1; echo "default rc=$?"; tail -3 $OUT/app_default.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 120 $A > $OUT/app_q16.log 2>&1; echo "q16 rc=$?"; tail -3 $OUT/app_q16.log
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 $A > $OUT/app_q8.log 2>&1; echo "q8 rc=$?"; tail -3 $OUT/app_q8.log
timeout -k 10 120 $A --device-mask 1 --counters > $OUT/app_counters.log 2>&1; echo "counters rc=$?"; tail -2 $OUT/app_counters.log
