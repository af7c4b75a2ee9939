#!/bin/bash
# one-pass top-k phase stamps; exactness; A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/bench_topk_phases.py --mode lsh > gpurun_out/d4_phases.jsonl 2> gpurun_out/d4_phases.err &&
timeout -k 10 120 python -u tools/bench_topk_phases.py --mode scores >> gpurun_out/d4_phases.jsonl 2>> gpurun_out/d4_phases.err &&
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_topk_scores.py tests/test_gpu_engines.py -k "topk or direct" > gpurun_out/d4_topk_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_topk_lsh.py --iters 200 > gpurun_out/d4_topk_lsh_ab.jsonl 2> gpurun_out/d4_topk_lsh_ab.err
