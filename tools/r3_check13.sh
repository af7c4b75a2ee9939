#!/bin/bash
# GMM EM with LDS-staged responsibilities: numerics, parity, throughput, kernel time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_native_clustering.py tests/test_gpu_engines.py -k "gmm or clustering" > gpurun_out/r3_c18_tests.log 2>&1 &&
timeout -k 10 200 python tools/bench_clustering.py --native --method gmm > gpurun_out/r3_cluster_native2.jsonl 2>/dev/null &&
timeout -k 10 200 python tools/bench_clustering.py --method gmm >> gpurun_out/r3_cluster_native2.jsonl 2>/dev/null &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cl2 -o cl -- python3 tools/bench_clustering.py --method gmm --points 50000 > gpurun_out/r3_prof_cl2.log 2>&1
