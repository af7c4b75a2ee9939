#!/bin/bash
# round-3 GPU check: serial-mode + native row-server tests, then the bench
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_scan.py tests/test_native_row_servers.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_serial_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
# a crash / timeout / fault (not a plain assertion failure, rc 1) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py --steps 10 --warmup 3 --no-rpc --engine-rows 300000 --lof-rows 20000 > gpurun_out/r3_bench_exact.json 2> gpurun_out/r3_bench_exact.err
echo "bench rc=$?"
