set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_gpu_engines.py tests/test_clustering.py tests/test_native_clustering.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5c/tests.log 2>&1; echo "tests rc=$?"
tail -2 gpurun_out/r5c/tests.log
timeout -k 10 300 python tools/bench_topk_mq.py > gpurun_out/r5c/mq_on7.jsonl 2>&1; echo "mq on rc=$?"
cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktq -o run -- python3 $R/tools/bench_topk_mq.py --quick --iters 10 > $R/gpurun_out/r5c/ktq.log 2>&1; echo "ktq rc=$?"
find /tmp/ktq -name "*kernel_stats*" -exec cp {} $R/gpurun_out/r5c/ \;
cd $R && tail -c 4000 gpurun_out/r5c/ktq.log > gpurun_out/r5c/ktq.tail && rm gpurun_out/r5c/ktq.log
bash tools/gpu_r5d.sh
