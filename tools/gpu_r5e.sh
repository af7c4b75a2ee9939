set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5e
timeout -k 10 600 python -u -m pytest tests/test_native_lof_batch.py tests/test_gpu_engines.py tests/test_native_row_dist_gpu.py tests/test_native_row_servers.py tests/test_native_clustering.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5e/tests.log 2>&1; echo "tests rc=$?"
tail -15 gpurun_out/r5e/tests.log
timeout -k 10 500 python tools/bench_engine_records.py --engines anomaly_lof,recommender_euclid_lsh,clustering_gmm,clustering_kmeans > gpurun_out/r5e/engines.json 2> gpurun_out/r5e/engines.err; echo "engines rc=$?"
tail -c 3000 gpurun_out/r5e/engines.json
timeout -k 10 300 python tools/bench_topk_mq.py > gpurun_out/r5e/mq_on7.jsonl 2>&1; echo "mq rc=$?"
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktq -o run -- python3 $R/tools/bench_topk_mq.py --quick --iters 10 > $R/gpurun_out/r5e/ktq.log 2>&1; echo "ktq rc=$?"
find /tmp/ktq -name "*kernel_stats*" -exec cp {} $R/gpurun_out/r5e/ \;
cd $R && tail -c 3000 gpurun_out/r5e/ktq.log > gpurun_out/r5e/ktq.tail && rm gpurun_out/r5e/ktq.log
timeout -k 10 200 python tools/prof_cluster.py --method gmm > gpurun_out/r5e/gmm.log 2>&1; echo "gmm rc=$?"
cat gpurun_out/r5e/gmm.log
