#!/bin/bash
# serial-mode per-batch cost (+ kernel profile) and the native row-server tests
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_serial.py --batches 60 > gpurun_out/r3_serial_batches.jsonl 2> gpurun_out/r3_serial_batches.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o prof -- python -u tools/bench_serial.py --batches 30 --modes exact > gpurun_out/r3_serial_prof.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_native_row_servers.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_rowsrv_tests.log 2>&1
echo "tests rc=$?"
