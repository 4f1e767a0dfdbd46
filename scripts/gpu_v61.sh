# v61: bench C3 per row-rotation variant (tile dispatch order experiment)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_bench_variants.sh v61bench C3
