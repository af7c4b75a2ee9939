#!/bin/bash
# exact-mode committer phase timings (tools/bench_serial.py diagnostics)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_serial.py --batches 200 --modes exact > gpurun_out/r3_serial4_batches.jsonl 2> gpurun_out/r3_serial4_batches.err
