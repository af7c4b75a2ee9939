#!/bin/bash
# PMC counters of the exact-mode committer (one pass each, own run per pass)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_serial
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_serial/trace -o run --output-format csv -- python3 tools/bench_serial.py --batches 40 --modes exact > gpurun_out/pmc_serial/trace.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmc_serial/p1 -o run --output-format csv -- python3 tools/bench_serial.py --batches 40 --modes exact > gpurun_out/pmc_serial/p1.log 2>&1
