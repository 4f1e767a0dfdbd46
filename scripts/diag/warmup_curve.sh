#!/bin/bash
# the driver's bench invocation, and the per-frame GPU time over the first frames
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-wu}; mkdir -p $OUT
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_like.log 2>&1; echo "rc=$?"
python -c "import json;l=[x for x in open('$OUT/driver_like.log') if x.startswith('{')][-1];d=json.loads(l);print('driver-like', d['ms_per_step'], d['roofline']['kernel_ms'], round(d['value']))"
timeout -k 10 200 python scripts/diag/frame_curve.py > $OUT/curve.log 2>&1; echo "curve rc=$?"; cat $OUT/curve.log
