#!/bin/bash
# The GPU suite with a heartbeat file (a long test is not taken for a hang by the runner's silence
# watchdog; pytest-timeout still ends a hung test after 300 s with its traceback), then smoke.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r03_s74}; mkdir -p $OUT
( while true; do date >> $OUT/heartbeat.log; sleep 30; done ) &
HB=$!
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
kill $HB
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log
