cd $GRAFT_REPO_ROOT
O=gpurun_out/v38c; mkdir -p $O
VRT_LIB=build/variants/libvrt_stamps.so timeout -k 10 300 python -u scripts/stamps.py --configs C3,C4 --slots 8192 --save $O > $O/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $O/stamps.log; [ $rc -eq 0 ] || exit $rc
rm build/variants/libvrt_stamps.so
timeout -k 10 400 python -u scripts/ab.py --rounds 8 --configs C1,C2,C3,C4 > $O/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.log | grep -v '^{'; [ $rc -eq 0 ] || exit $rc
