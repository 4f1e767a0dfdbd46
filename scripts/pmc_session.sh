#!/bin/bash
# PMC collection for the render kernel (one counter group per rocprofv3 pass).
# Usage: bash scripts/pmc_session.sh <tag> [config]
TAG=${1:-pmc}; CFG=${2:-C3}
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $GROUP -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --config "$CFG" --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($GROUP) rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32
GROUPS
exit 0
