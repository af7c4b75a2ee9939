set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_linear.py -m gpu -x -v --timeout 300 --timeout-method thread -k "serial" > gpurun_out/t_serial.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python tools/bench_serial.py --batches 40 --modes exact > gpurun_out/serial_v.log 2>&1 && \
JB_SERIAL_COMMITTER=delta timeout -k 10 300 python tools/bench_serial.py --batches 40 --modes exact > gpurun_out/serial_d.log 2>&1
echo "bench rc=$?"
