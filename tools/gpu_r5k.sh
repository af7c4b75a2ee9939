set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py -q -m gpu --timeout 120 --timeout-method thread -k "one_launch_path" > gpurun_out/r5k/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5k/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/bench_topk_lsh.py --rows 100000 --iters 200 --cases 1:10,4:10,1:31,4:40,1:94 --paths select,default --metrics 1,0 > gpurun_out/r5k/topk_100k.jsonl 2>&1 || exit 1
cat gpurun_out/r5k/topk_100k.jsonl
timeout -k 10 200 python tools/bench_topk_lsh.py --rows 1000000 --iters 100 --cases 1:10,4:10,1:31,4:40,1:100 --paths select,default --metrics 1 > gpurun_out/r5k/topk_1m.jsonl 2>&1 || exit 1
cat gpurun_out/r5k/topk_1m.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5k/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_topk_lsh.py --rows 100000 --iters 100 --cases 1:31,4:40 --paths select,default --metrics 1 > $GRAFT_REPO_ROOT/gpurun_out/r5k/prof.log 2>&1; echo "prof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/r5k/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/r5k/kstats.csv
cut -d, -f1-8 $GRAFT_REPO_ROOT/gpurun_out/r5k/kstats.csv | head -12
rm -rf $GRAFT_REPO_ROOT/gpurun_out/r5k/prof
