set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py -m gpu -x -q --timeout 300 --timeout-method thread -k "serial" > gpurun_out/t_serial.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/t_serial.log
JB_COMMIT_PROF=1 timeout -k 10 200 python tools/bench_serial.py --batches 30 --modes exact > gpurun_out/serial_prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 200 python tools/bench_serial.py --batches 40 --modes exact > gpurun_out/serial_v.log 2>&1
echo "v rc=$?"
JB_COMMIT_PROF=1 timeout -k 10 200 python tools/bench_serial.py --batches 4 --modes exact --worst-case > gpurun_out/serial_profw.log 2>&1
echo "profw rc=$?"
