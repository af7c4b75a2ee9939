set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_native_row_servers.py -q -m gpu --timeout 120 --timeout-method thread -k "pool or recommender or inverted" > gpurun_out/r5s/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r5s/tests.log; [ $rc -eq 0 ] || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5sprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_engine_records.py --engines recommender_default > $GRAFT_REPO_ROOT/gpurun_out/r5s/prof.log 2>&1; echo "prof rc=$?"
cp /tmp/r5sprof/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/r5s/kstats.csv && cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/r5s/kstats.csv | cut -c1-120 | head -8
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/bench_engine_records.py --engines recommender_default > gpurun_out/r5s/eng.json 2>gpurun_out/r5s/eng.err; echo "eng rc=$?"; cut -c1-900 gpurun_out/r5s/eng.json
