#!/bin/bash
# The round's headline numbers in one call: bench.py at every config (default 500-after-200 shape,
# and the driver's 20-after-5 at C3), textured C3/C4, and the one-GPU strong-scaling rehearsal of
# C3/C4 at k = 1, 2, 4, 8 in both shapes. Usage: bash scripts/gpu_numbers.sh TAG
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/${1:-numbers}; mkdir -p $OUT
b() {  # b <name> <args...>
  local name=$1; shift
  timeout -k 10 200 python bench.py --cpu-seconds 0 "$@" > $OUT/$name.log 2>&1 || exit $?
  python - "$OUT/$name.log" "$name" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]
d = json.loads(l)
print(sys.argv[2], d['ms_per_step'], round(d['value']), d.get('kernel_ms'), d.get('verified'))
PY
}
for cfg in C1 C2 C3 C4; do b bench_$cfg --config $cfg; done
b drv_C3 --config C3 --steps 20 --warmup 5
b tex_C3 --config C3 --shading textured
b tex_C4 --config C4 --shading textured
for cfg in C3 C4; do for k in 1 2 4 8; do
  b rh_${cfg}_k${k}_steady --config $cfg --rehearse-ranks $k --steps 500 --warmup 200 --no-verify
  b rh_${cfg}_k${k}_drv --config $cfg --rehearse-ranks $k --steps 20 --warmup 5 --no-verify
done; done
