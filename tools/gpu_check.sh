#!/bin/bash
# GPU-box check: the GPU test tier, then a short headline bench (outputs under gpurun_out/)
# usage: tools/gpu_check.sh TAG [pytest selection...]
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-check}
shift
SEL=${*:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
