#!/bin/bash
# headless app frame times: synchronous (per-frame GPU time) and pipelined (display path)
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-diag}; mkdir -p $OUT
A="build/bin/vrt_headless --scene ${SCENE:-refraction} --n ${N:-128} --size ${SIZE:-1920x1080} --bounces ${BOUNCES:-4 4} --frames 400 --warmup 200 --quiet"
timeout -k 10 120 $A > $OUT/app_sync.log 2>&1; echo "sync rc=$?"; tail -1 $OUT/app_sync.log
timeout -k 10 120 $A --pipelined > $OUT/app_pipe.log 2>&1; echo "pipelined rc=$?"; tail -1 $OUT/app_pipe.log
timeout -k 10 200 python bench.py --config ${CFG:-C3} --steps 200 --warmup 200 --cpu-seconds 0 --no-verify > $OUT/bench.log 2>&1; echo "bench rc=$?"
python -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('bench', d['roofline']['kernel_ms'])"
