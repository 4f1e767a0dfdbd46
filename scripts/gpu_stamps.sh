cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
VRT_LIB=build/variants/libvrt_stamps.so timeout -k 10 300 python -u scripts/stamps.py --configs ${2:-C1,C2,C3,C4} --slots 8192 --save $O > $O/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $O/stamps.log; exit $rc
