cd $GRAFT_REPO_ROOT
O=gpurun_out/v36; mkdir -p $O/deep; export TMPDIR=/tmp
bash scripts/pmc_deep.sh gpurun_out/v36/deep C3 C4 || exit 1
ls $O/deep
