#!/bin/bash
# exact mode (cheap |x|_1 Dmax bound) + device DF kernel tests, then exact-mode batches
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_fv_wide.py tests/test_gpu_engines.py -m gpu -k "serial or deviation or wide or gmm or clustering" > gpurun_out/r3_c12_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_serial.py --batches 160 --modes exact > gpurun_out/r3_serial11_batches.jsonl 2> gpurun_out/r3_serial11_batches.err
