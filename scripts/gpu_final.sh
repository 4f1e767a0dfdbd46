#!/bin/bash
# Round-end evidence in one call: GPU suite + smoke + bench + rocprofv3 trace/PMC of C3 (stamped
# with the library hash), every config's bench line (textured C3/C4 too), then the strong-scaling
# rehearsal table over every rank.
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r03_s56}
bash scripts/gpu_check.sh $TAG C3 || exit $?
OUT=gpurun_out/${TAG}_all; mkdir -p $OUT
for spec in "C1 color" "C2 color" "C4 color" "C3 textured" "C4 textured"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --shading $2 --cpu-seconds 0 > $OUT/bench_$1_$2.log 2>&1 || exit 1
  python -c "import json;l=[x for x in open('$OUT/bench_$1_$2.log') if x.startswith('{')][-1];d=json.loads(l);print('$1 $2', d['ms_per_step'], d['config'].get('hw_queues'), round(d['value']), d['verified'])"
done
bash scripts/diag/strong_table.sh ${TAG}_strong
