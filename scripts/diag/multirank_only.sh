#!/bin/bash
# The two-rank bench rehearsal tests alone, verbose, with a heartbeat.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s75}; mkdir -p $OUT
( while true; do date >> $OUT/heartbeat.log; sleep 30; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
kill $HB
grep -E "PASSED|FAILED|Timeout" $OUT/pytest.log | head -5
exit $rc
