#!/bin/bash
# the driver's 1-GPU bench (defaults), JSON line + progress log
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 840 python -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
