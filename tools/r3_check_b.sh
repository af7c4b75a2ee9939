#!/bin/bash
# bf16 W tests; one-launch top-k tests + A/B; regression; smoke; bench with the bf16 record
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16.py > gpurun_out/r3_bf16_tests.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_topk_scores.py tests/test_gpu_engines.py -k "topk or direct" > gpurun_out/r3_topk_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_topk_scores.py --iters 200 > gpurun_out/r3_topk_ab.jsonl 2> gpurun_out/r3_topk_ab.err &&
timeout -k 10 300 python -u tools/bench_topk_lsh.py --iters 200 > gpurun_out/r3_topk_lsh_ab.jsonl 2> gpurun_out/r3_topk_lsh_ab.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r3_all_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-rpc --engines none --exact-steps 0 > gpurun_out/r3_bench_bf16.log 2>&1
