set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5p
bash tools/gpu_session.sh tests smoke
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5pprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_engine_records.py --engines recommender_default > $GRAFT_REPO_ROOT/gpurun_out/r5p/prof.log 2>&1; echo "prof rc=$?"
cp /tmp/r5pprof/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/r5p/kstats.csv && cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/r5p/kstats.csv | cut -c1-120 | head -12
tail -c 1500 $GRAFT_REPO_ROOT/gpurun_out/r5p/prof.log
