#!/bin/bash
# exact mode (plain-store steps) tests + batches; clustering push on the GPU
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_engines.py tests/test_clustering.py -k "serial or deviation or gmm or clustering" > gpurun_out/r3_c14_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_clustering.py --points 200000 --method kmeans > gpurun_out/r3_cluster2.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/bench_clustering.py --points 200000 --method gmm >> gpurun_out/r3_cluster2.jsonl 2>&1 &&
timeout -k 10 400 python -u tools/bench_serial.py --batches 160 --modes exact > gpurun_out/r3_serial13_batches.jsonl 2> gpurun_out/r3_serial13_batches.err
