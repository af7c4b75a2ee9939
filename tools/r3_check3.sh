#!/bin/bash
# exact-mode v2: correctness tests, per-batch cost, kernel profile
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_scan.py -m gpu -q -k "serial or concurrent or arena" --timeout 150 --timeout-method thread > gpurun_out/r3_serial2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_serial.py --batches 60 > gpurun_out/r3_serial2_batches.jsonl 2> gpurun_out/r3_serial2_batches.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_serial2 -o prof -- python -u $GRAFT_REPO_ROOT/tools/bench_serial.py --batches 30 --modes exact > $GRAFT_REPO_ROOT/gpurun_out/r3_serial2_prof.log 2>&1
