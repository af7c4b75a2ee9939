set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5n
timeout -k 10 600 python -u -m pytest tests/test_lof_state.py tests/test_native_lof_batch.py tests/test_native_row_servers.py tests/test_native_row_dist_gpu.py tests/test_lof_mix.py -q -m gpu --timeout 120 --timeout-method thread -k "lof or anomaly" > gpurun_out/r5n/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5n/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_engine_records.py --engines anomaly_lof > gpurun_out/r5n/eng.json 2>gpurun_out/r5n/eng.err; echo "eng rc=$?"; cut -c1-1500 gpurun_out/r5n/eng.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5nprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_engine_records.py --engines anomaly_lof > $GRAFT_REPO_ROOT/gpurun_out/r5n/prof.log 2>&1; echo "prof rc=$?"
cp /tmp/r5nprof/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/r5n/kstats.csv && cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/r5n/kstats.csv | cut -c1-120 | head -8
