set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
timeout -k 10 900 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_topk_scores.py tests/test_lof_state.py tests/test_native_lof_batch.py tests/test_native_row_servers.py tests/test_native_row_dist_gpu.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5l/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5l/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_engine_records.py --engines anomaly_lof,recommender_euclid_lsh > gpurun_out/r5l/eng.json 2>gpurun_out/r5l/eng.err; echo "eng rc=$?"; cut -c1-2500 gpurun_out/r5l/eng.json
timeout -k 10 200 python tools/bench_topk_lsh.py --rows 100000 --iters 200 --cases 1:10,4:10,1:31,4:40,1:94 --paths select,default --metrics 1,0 > gpurun_out/r5l/topk_100k.jsonl 2>&1 || exit 1
cat gpurun_out/r5l/topk_100k.jsonl
timeout -k 10 300 python tools/bench_topk_scores.py --rows 1000000 --iters 100 --paths chain,fused,select,default > gpurun_out/r5l/scores_1m.jsonl 2>&1 || exit 1
cat gpurun_out/r5l/scores_1m.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5lprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_topk_lsh.py --rows 100000 --iters 100 --cases 1:10,1:31,4:40 --paths select,default --metrics 1 > $GRAFT_REPO_ROOT/gpurun_out/r5l/prof.log 2>&1; echo "prof rc=$?"
find /tmp/r5lprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/r5l/kstats.csv
cut -d, -f1-8 $GRAFT_REPO_ROOT/gpurun_out/r5l/kstats.csv | cut -c1-200 | head -14
