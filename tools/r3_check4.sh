#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_serial.py --batches 400 --modes exact,atomic > gpurun_out/r3_serial3_batches.jsonl 2> gpurun_out/r3_serial3_batches.err
