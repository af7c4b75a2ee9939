#!/bin/bash
# session-4 final check: full GPU suite (no -x: every failure in one pass), smoke, default bench
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3s5_gpu_tests.log 2>&1
rc=$?
# 0 = all passed, 1 = some tests failed: anything else (abort, timeout, crash) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s5_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r3s5_bench.log 2>&1 || exit $?
exit $rc
