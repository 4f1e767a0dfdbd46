#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-parts}; mkdir -p $OUT
for cfg in C3 C2 C4; do for p in 1 2 3 4; do
  timeout -k 10 200 python bench.py --config $cfg --parts $p --cpu-seconds 0 --no-verify > $OUT/${cfg}_p$p.log 2>&1 || exit $?
  python -c "import json;l=[x for x in open('$OUT/${cfg}_p$p.log') if x.startswith('{')][-1];d=json.loads(l);print('$cfg parts $p', d['ms_per_step'])"
done; done
