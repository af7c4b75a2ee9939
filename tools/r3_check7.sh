#!/bin/bash
# native distributed classifier (GPU) + exact-mode per-wave committer timings
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_native_dist_gpu.py > gpurun_out/r3_c10_dist.log 2>&1
rc=$?
cp /tmp/native_dist_*.log gpurun_out/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_serial.py --batches 160 --modes exact > gpurun_out/r3_serial9_batches.jsonl 2> gpurun_out/r3_serial9_batches.err
