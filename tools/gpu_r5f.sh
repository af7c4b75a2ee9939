set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5f
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_native_clustering.py tests/test_clustering.py tests/test_native_lof_batch.py tests/test_gpu_linear.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5f/tests.log 2>&1; echo "tests rc=$?"
tail -15 gpurun_out/r5f/tests.log
timeout -k 10 500 python tools/bench_engine_records.py --engines anomaly_lof,recommender_euclid_lsh,clustering_gmm,clustering_kmeans > gpurun_out/r5f/engines.json 2> gpurun_out/r5f/engines.err; echo "engines rc=$?"
tail -c 3000 gpurun_out/r5f/engines.json
timeout -k 10 200 python tools/prof_cluster.py --method gmm > gpurun_out/r5f/gmm.log 2>&1; echo "gmm rc=$?"
cat gpurun_out/r5f/gmm.log
