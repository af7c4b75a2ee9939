#!/bin/bash
# native distributed MIX at the default (2^24) and a 2^20 table; fixed tests; top-k path A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_native_dist_gpu.py -k distributed_mix > gpurun_out/d1_dist24.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
JUBATUS_DEVICE_HASH_BITS=20 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_native_dist_gpu.py -k distributed_mix > gpurun_out/d1_dist20.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_native_server_gpu.py tests/test_gpu_bf16.py > gpurun_out/d1_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_topk_lsh.py --iters 200 > gpurun_out/d1_topk_lsh_ab.jsonl 2> gpurun_out/d1_topk_lsh_ab.err &&
timeout -k 10 300 python -u tools/bench_topk_scores.py --iters 200 > gpurun_out/d1_topk_scores_ab.jsonl 2> gpurun_out/d1_topk_scores_ab.err
