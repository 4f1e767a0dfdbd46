#!/bin/bash
# Cache / memory-latency PMC passes (one rocprofv3 --pmc run per group, kernel trace only) over
# the bench's C3 frame: L2 hit rate, vL1D accesses, TA busy, mean VMEM latency
# (SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM_RD). Usage: bash scripts/pmc_cache.sh OUTDIR CFG...
out=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); export TMPDIR=/tmp
mkdir -p "$ROOT/$out"
timeout -k 10 60 rocprofv3 -L > "$ROOT/$out/avail.txt" 2>&1 || true
for cfg in "$@"; do
  i=0
  for grp in "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVES SQ_WAVE_CYCLES" \
             "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp -d "$ROOT/$out/${cfg}_c$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 0 --device-warmup-ms 0 > "$ROOT/$out/${cfg}_c$i.log" 2>&1
    rc=$?; echo "$cfg group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
