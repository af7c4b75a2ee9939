#!/bin/bash
# exact-mode check after the re-scored segments: per-batch costs, then a kernel-time profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python -u tools/bench_serial.py --batches 60 --modes exact > gpurun_out/r3s4_serial_batches.jsonl 2> gpurun_out/r3s4_serial.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial4 -o ser -- python3 tools/bench_serial.py --batches 40 --modes exact > gpurun_out/r3s4_serial_prof.log 2>&1
