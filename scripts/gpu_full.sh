#!/bin/bash
# Full check of a build: GPU suite, smoke, driver-shaped and default benches, strong-scaling
# rehearsal (K = 1, 2, 4, 8), kernel trace of the default bench. Stops at a fault / timeout.
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-r03_full}; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum voxelraytracer_amd/_lib/libvrt.so | cut -d" " -f1 > $OUT/lib.sha256
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"verified": [a-z]*' $OUT/$name.log | head -3 | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
[ -n "$SKIP_TESTS" ] || step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[ -n "$SKIP_TESTS" ] || step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step drv_C3 300 python bench.py --steps 20 --warmup 5
step bench_C3 300 python bench.py
for cfg in C3 C4; do for k in 1 2 4 8; do
  step rh_${cfg}_k${k}_drv 200 python bench.py --config $cfg --rehearse-ranks $k --steps 20 --warmup 5 --cpu-seconds 0 --no-verify
  step rh_${cfg}_k${k} 200 python bench.py --config $cfg --rehearse-ranks $k --cpu-seconds 0 --no-verify
done; done
step bench_C3_tex 300 python bench.py --shading textured --cpu-seconds 0
step trace_C3 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" --cpu-seconds 0
exit 0
