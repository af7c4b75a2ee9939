#!/bin/bash
# per-kernel time of the native clustering server (gmm push bench)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cl -o cl -- python3 tools/bench_clustering.py --method gmm --points 50000 > gpurun_out/r3_prof_cl.log 2>&1
