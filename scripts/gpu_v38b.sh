cd $GRAFT_REPO_ROOT
O=gpurun_out/v38b; mkdir -p $O
VRT_LIB=build/variants/libvrt_certdiag.so timeout -k 10 200 python -u scripts/cert_diag.py > $O/cert_diag.log 2>&1; rc=$?; grep -v amdgpu.ids $O/cert_diag.log; [ $rc -eq 0 ] || exit $rc
rm build/variants/libvrt_certdiag.so
timeout -k 10 400 python -u scripts/ab.py --rounds 8 --configs C1,C2,C3,C4 > $O/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.log | grep -v '^{'; [ $rc -eq 0 ] || exit $rc
