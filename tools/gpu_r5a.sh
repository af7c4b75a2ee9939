set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for sh in r1pd2 r1pd1 r1pd3 r2pd1 r2pd2; do
  JB_VC_SHAPE=$sh timeout -k 10 200 python tools/bench_serial.py --batches 30 --modes exact > gpurun_out/serial_$sh.log 2>&1
  echo "$sh rc=$?"; tail -1 gpurun_out/serial_$sh.log | cut -c1-200
done
JB_VC_SHAPE=r1pd2 timeout -k 10 300 python tools/bench_serial.py --batches 6 --modes exact --worst-case > gpurun_out/serial_vw.log 2>&1
echo "worst rc=$?"
