set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk_scores.py tests/test_lof_state.py tests/test_native_lof_batch.py tests/test_native_row_servers.py tests/test_native_row_dist_gpu.py tests/test_gpu_engines.py -q -m gpu --timeout 120 --timeout-method thread -k "lof or anomaly or scores or row" > gpurun_out/r5m/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5m/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python tools/bench_engine_records.py --engines anomaly_lof,recommender_default,recommender_euclid_lsh > gpurun_out/r5m/eng.json 2>gpurun_out/r5m/eng.err; echo "eng rc=$?"; cut -c1-3000 gpurun_out/r5m/eng.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5mprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_engine_records.py --engines anomaly_lof > $GRAFT_REPO_ROOT/gpurun_out/r5m/prof.log 2>&1; echo "prof rc=$?"
find /tmp/r5mprof -name "*kernel_stats.csv" | xargs ls -la | head
for f in $(find /tmp/r5mprof -name "*kernel_stats.csv"); do n=$(basename $(dirname $f)); cp $f $GRAFT_REPO_ROOT/gpurun_out/r5m/kstats_$n.csv; done
for f in $GRAFT_REPO_ROOT/gpurun_out/r5m/kstats_*.csv; do echo $f; cut -d, -f1-4 $f | cut -c1-150 | head -12; done
