cd $GRAFT_REPO_ROOT
O=gpurun_out/v46; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cert.log 2>&1; rc=$?; tail -3 $O/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
VRT_LIB=build/variants/libvrt_certdiag.so timeout -k 10 200 python -u scripts/cert_diag.py > $O/cert_diag.log 2>&1; rc=$?; grep -v amdgpu.ids $O/cert_diag.log; [ $rc -eq 0 ] || exit $rc
rm build/variants/libvrt_certdiag.so
bash scripts/gpu_ab.sh v46ab C1,C2,C3,C4 && bash scripts/gpu_bench_variants.sh v46bench C3 C1
