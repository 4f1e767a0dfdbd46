#!/bin/bash
# PMC of the stats-free render kernel for several libraries (VRT_LIB), one rocprofv3 --pmc run per
# counter group: bash scripts/pmc_variants.sh OUTDIR CFG LIB...   (LIB = path or "base")
set -e
out=$1; cfg=$2; shift 2; mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "$lib" .so)
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    if [ "$lib" = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
    timeout -k 10 120 rocprofv3 --pmc $grp -d "$ROOT/$out/${name}_${cfg}_g$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 0 --parts 1 > "$ROOT/$out/${name}_${cfg}_g$i.log" 2>&1
  done
done
unset VRT_LIB
