set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engines.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_eng.log 2>&1 || { tail -30 gpurun_out/gpu_eng.log; exit 1; }
tail -2 gpurun_out/gpu_eng.log
timeout -k 10 200 python tools/bench_topk.py > gpurun_out/topk16.json
JB_TOPK_MERGE=tile timeout -k 10 300 python tools/bench_engines.py recommender > gpurun_out/engines_mt.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_topk16 -o topk -- python3 tools/bench_topk.py > /dev/null 2>&1
JB_TOPK_MERGE=tile timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_topkmt -o topk -- python3 tools/bench_topk.py > /dev/null 2>&1
timeout -k 10 300 python tools/bench_engines.py recommender anomaly > gpurun_out/engines.jsonl 2> gpurun_out/engines.err
cat gpurun_out/engines.jsonl
