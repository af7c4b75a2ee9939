#!/bin/bash
# exact mode: serial-equivalence tests, then per-batch cost with committer phases
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py -k "serial or deviation" > gpurun_out/r3_c8_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_serial.py --batches 160 --modes exact > gpurun_out/r3_serial7_batches.jsonl 2> gpurun_out/r3_serial7_batches.err
