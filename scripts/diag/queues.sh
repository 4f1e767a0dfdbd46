#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-q}; mkdir -p $OUT
A="build/bin/vrt_headless --scene refraction --n 128 --size 1920x1080 --bounces 4 4 --frames 600 --warmup 300 --quiet --pipelined"
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --cpu-seconds 0 --no-verify > $OUT/bench_q$q.log 2>&1 || exit $?
  python -c "import json;l=[x for x in open('$OUT/bench_q$q.log') if x.startswith('{')][-1];d=json.loads(l);print('bench queues $q', d['ms_per_step'])"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 $A > $OUT/app_q$q.log 2>&1 || exit $?; echo "app queues $q: $(tail -1 $OUT/app_q$q.log)"
done
