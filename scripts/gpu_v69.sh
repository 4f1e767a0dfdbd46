# v69: A/B of the bounce-stack code layout (noinline march_cert / air segment) and 6 waves/SIMD
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh v69ab C1,C2,C3,C4
