set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5b
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ktv -o run -- python3 $R/tools/bench_serial.py --batches 30 --modes exact > $R/gpurun_out/r5b/ktv.log 2>&1; echo "ktv rc=$?"
cd $R && python3 tools/trace_gaps.py /tmp/ktv gpurun_out/r5b/gaps_steady.md --last 1500 > /dev/null && python3 tools/trace_gaps.py /tmp/ktv gpurun_out/r5b/gaps_all.md > /dev/null; echo "gaps rc=$?"
cd /tmp
JB_SERIAL_COMMITTER=delta timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/dw -o run -- python3 $R/tools/bench_serial.py --batches 3 --modes exact > $R/gpurun_out/r5b/delta_write.log 2>&1; echo "delta write rc=$?"
cd $R
for f in gpurun_out/r5b/*.log; do tail -c 20000 $f > $f.t && mv $f.t $f; done
