set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r03_s5; mkdir -p $OUT
timeout -k 10 300 python -u scripts/diag/host_rate.py > $OUT/host_rate.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame_api.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_frame_api.log 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for cfg in C3 C4; do for k in 1 2 4 8; do
  for shape in "--steps 20 --warmup 5" "--steps 500 --warmup 200"; do
    timeout -k 10 200 python bench.py --config $cfg --rehearse-ranks $k $shape --cpu-seconds 0 --no-verify > $OUT/rh_${cfg}_k${k}_$(echo $shape | tr -d ' -').log 2>&1 || exit $?
  done
done; done
exit $rc
