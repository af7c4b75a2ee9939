#!/bin/bash
# full GPU test suite + smoke + clustering push rates (in process and over RPC)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 &&
for m in kmeans gmm; do
  timeout -k 10 200 python tools/bench_clustering.py --method $m >> gpurun_out/r3_cluster.jsonl 2>/dev/null &&
  timeout -k 10 200 python tools/bench_clustering.py --native --method $m >> gpurun_out/r3_cluster.jsonl 2>/dev/null || exit 1
done
