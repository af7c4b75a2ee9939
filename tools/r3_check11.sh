#!/bin/bash
# native jubaclustering parity on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_native_clustering.py > gpurun_out/r3_c15_tests.log 2>&1
