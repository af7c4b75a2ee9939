set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5h
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_engines.py -q -m gpu --timeout 120 --timeout-method thread -k "serial or gmm or kmeans or exact" > gpurun_out/r5h/tests.log 2>&1; echo "tests rc=$?"
tail -5 gpurun_out/r5h/tests.log
timeout -k 10 300 python tools/bench_serial.py --batches 40 --modes exact > gpurun_out/r5h/serial.log 2>&1; echo "serial rc=$?"
grep "^{" gpurun_out/r5h/serial.log | cut -c1-400
timeout -k 10 200 python tools/prof_cluster.py --method gmm > gpurun_out/r5h/gmm.log 2>&1; echo "gmm rc=$?"
cat gpurun_out/r5h/gmm.log
