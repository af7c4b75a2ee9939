#!/bin/bash
# GPU-box check: the GPU test tier, then a short headline bench (outputs under gpurun_out/)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1d.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_r1d.json 2> gpurun_out/bench_r1d.err
