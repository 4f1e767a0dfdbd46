# usage: bash scripts/gpu_ab.sh OUTDIR [CONFIGS]  -- interleaved A/B of build/variants against the default lib
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u scripts/ab.py --rounds 8 --configs ${2:-C1,C2,C3,C4} > $O/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.log | grep -v '^{'; exit $rc
