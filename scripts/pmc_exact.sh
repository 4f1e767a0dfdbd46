#!/bin/bash
# One rocprofv3 PMC pass over the C3 bench with the exact pass's instruction-mix counters
# (scratch, vector-memory reads/writes, LDS, waits), after checking every counter name against
# `rocprofv3 -L` on this box. Usage: bash scripts/pmc_exact.sh TAG [CFG]
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); TAG=$1; CFG=${2:-C3}; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
want="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_SCRATCH"
have=""
for c in $want; do grep -qw "$c" $OUT/avail.txt && have="$have $c"; done
echo "counters:$have"
[ -n "$have" ] || exit 1
set -- $have; [ $# -le 8 ] || exit 1
timeout -s KILL 120 rocprofv3 --pmc $have -d $OUT/pmc_mix -o run --output-format csv -- \
  python3 $ROOT/bench.py --config $CFG --steps 5 --warmup 1 --cpu-seconds 0 --parts 1 --no-verify > $OUT/pmc_mix.log 2>&1
echo "rc=$?"
