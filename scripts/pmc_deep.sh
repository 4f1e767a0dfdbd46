#!/bin/bash
# Extra PMC passes (one rocprofv3 --pmc run per counter group, kernel trace only): VALU lane
# utilisation, VMEM latency, LDS waits/conflicts. Usage: bash scripts/pmc_deep.sh OUTDIR CFG...
set -e
out=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); export TMPDIR=/tmp; mkdir -p "$ROOT/$out"
for cfg in "$@"; do
  i=0
  for grp in "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp -d "$ROOT/$out/${cfg}_g$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 0 --parts 1 > "$ROOT/$out/${cfg}_g$i.log" 2>&1
  done
done
