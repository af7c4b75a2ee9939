#!/bin/bash
# bf16 W storage: numerics vs the fp32 oracle, HBM-sized table MIX, linear regression check, bench record
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/r3_bf16_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_linear.py tests/test_native_server_gpu.py tests/test_gpu_server.py > gpurun_out/r3_linear_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-rpc --engines none --exact-steps 0 > gpurun_out/r3_bench_bf16.log 2>&1
