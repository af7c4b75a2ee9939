#!/bin/bash
# round-3 kernel profiles: train pipeline (atomic + one exact step), LSH top-k at 10M rows
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train3 -o tr -- python3 bench.py --steps 3 --warmup 1 --no-rpc --engines none --exact-steps 1 --bf16-steps 0 --worst-steps 0 --batches-per-step 8 > gpurun_out/p3_train.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_topk_lsh.py --rows 10000000 --iters 50 > gpurun_out/p3_lsh10m.jsonl 2> gpurun_out/p3_lsh10m.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lsh10m -o lsh -- python3 tools/bench_topk_lsh.py --rows 10000000 --iters 20 > gpurun_out/p3_lsh10m_prof.log 2>&1
