set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 600 python -u -m pytest tests/test_lof_state.py tests/test_native_lof_batch.py tests/test_gpu_engines.py tests/test_native_row_servers.py tests/test_lof_mix.py -q -m gpu --timeout 120 --timeout-method thread -k "lof or anomaly or one_launch_path" > gpurun_out/r5j/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5j/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_engine_records.py --engines anomaly_lof > gpurun_out/r5j/lof.json 2>gpurun_out/r5j/lof.err; echo "lof rc=$?"; cut -c1-1500 gpurun_out/r5j/lof.json
timeout -k 10 200 python tools/bench_topk_lsh.py --rows 100000 --iters 200 --cases 1:10,1:31,4:40,1:94 --paths fused,select,default --metrics 1,0 > gpurun_out/r5j/topk_100k.jsonl 2>&1 || exit 1
cat gpurun_out/r5j/topk_100k.jsonl
timeout -k 10 200 python tools/bench_topk_lsh.py --rows 1000000 --iters 100 --cases 1:10,1:31,4:40,1:100 --paths fused,select,default --metrics 1 > gpurun_out/r5j/topk_1m.jsonl 2>&1 || exit 1
cat gpurun_out/r5j/topk_1m.jsonl
