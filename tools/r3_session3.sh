#!/bin/bash
# session-3 check: full GPU suite, smoke, default bench (driver contract)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s3_gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s3_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r3s3_bench.log 2>&1
