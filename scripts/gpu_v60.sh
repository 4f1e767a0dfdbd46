# v60: per-axis jump limit: certified suite, wave timeline, bench C1-C4
cd $GRAFT_REPO_ROOT
O=gpurun_out/v60; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_certified.py -x -q --timeout 120 --timeout-method thread > $O/pytest_cert.log 2>&1; rc=$?; tail -2 $O/pytest_cert.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_v59.sh || exit $?
rm -f build/variants/libvrt_stamps.so
for c in C1 C2 C3 C4; do timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 > $O/bench_$c.log 2>&1 || exit 1; echo "$c $(tail -1 $O/bench_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
