#!/bin/bash
# one-pass top-k: exactness tests, path A/B, kernel trace of the A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_topk_scores.py tests/test_gpu_engines.py -k "topk or direct" > gpurun_out/d3_topk_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_topk_lsh.py --iters 200 > gpurun_out/d3_topk_lsh_ab.jsonl 2> gpurun_out/d3_topk_lsh_ab.err &&
timeout -k 10 300 python -u tools/bench_topk_scores.py --iters 200 > gpurun_out/d3_topk_scores_ab.jsonl 2> gpurun_out/d3_topk_scores_ab.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_topk3 -o tk -- python3 tools/bench_topk_lsh.py --iters 50 > gpurun_out/d3_prof.log 2>&1
