# v71: heavy tiles at raised wave priority from their start (bench C3 per variant)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_bench_variants.sh v71bench C3 C3
