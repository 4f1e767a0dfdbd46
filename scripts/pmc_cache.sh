#!/bin/bash
# L2 hit/miss of the render kernel per library: bash scripts/pmc_cache.sh OUTDIR CFG LIB...
set -e
out=$1; cfg=$2; shift 2; mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "$lib" .so)
  if [ "$lib" = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$ROOT/$out/${name}_${cfg}_g1" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 0 --parts 1 > "$ROOT/$out/${name}_${cfg}_g1.log" 2>&1
done
unset VRT_LIB
