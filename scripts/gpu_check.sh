#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel trace + PMC passes.
# Usage (on the box): bash scripts/gpu_check.sh [tag] [config]
# Stops at the first step that is not a clean pass/fail (fault, abort, timeout).
TAG=${1:-run}; CFG=${2:-C3}
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
sha256sum voxelraytracer_amd/_lib/libvrt.so | cut -d" " -f1 > "$OUT/lib.sha256"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  ok $rc || exit $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 300 python bench.py --config "$CFG"
export TMPDIR=/tmp
# the bench command itself under the kernel trace (its JSON line lands in prof_trace.log): the
# bench's launch_ms and rocprofv3's mean kernel duration come from the same process
step prof_trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CFG" --cpu-seconds 0
[ -n "$NO_PMC" ] && exit 0
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --device-warmup-ms 0
step prof_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --device-warmup-ms 0
step prof_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 1 --cpu-seconds 0 --device-warmup-ms 0
exit 0
