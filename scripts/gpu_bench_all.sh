#!/bin/bash
# bench.py on every GPU config (no CPU leg) + the headless C++ host's frame times at C3
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-ball}; mkdir -p $OUT
for cfg in C1 C2 C3 C4; do
  timeout -k 10 200 python bench.py --config $cfg --cpu-seconds 0 > $OUT/bench_$cfg.log 2>&1 || exit $?
  python -c "import json;l=[x for x in open('$OUT/bench_$cfg.log') if x.startswith('{')][-1];d=json.loads(l);print('$cfg', d['ms_per_step'], round(d['value']), d['verified'])"
done
bash scripts/diag_app.sh ${1:-ball}_app
