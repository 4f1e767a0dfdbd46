# v66: reproducibility of the tile-order bench (C3 twice per library)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_bench_variants.sh v66bench C3 C3
