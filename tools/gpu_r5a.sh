set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/pmc5
JB_COMMIT_PROF=1 timeout -k 10 200 python tools/bench_serial.py --batches 30 --modes exact > gpurun_out/serial_prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 200 python tools/bench_serial.py --batches 40 --modes exact > gpurun_out/serial_v.log 2>&1
echo "v rc=$?"
cd /tmp
B="python3 $R/tools/bench_serial.py --batches 6 --modes exact,atomic"
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d /tmp/pw -o run -- $R/tools/probes/lds_pmc_probe > $R/gpurun_out/pmc5/probe_w.log 2>&1; echo "probe write rc=$?"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o run -- $B > $R/gpurun_out/pmc5/kt.log 2>&1; echo "kt rc=$?"
find /tmp/kt -name "*stats*" -exec cp {} $R/gpurun_out/pmc5/ \; ; find /tmp/kt -type f > $R/gpurun_out/pmc5/kt_files.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --kernel-trace --output-format csv -d /tmp/sq1 -o run -- $B > $R/gpurun_out/pmc5/sq1.log 2>&1; echo "sq1 rc=$?"
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-trace --output-format csv -d /tmp/sq2 -o run -- $B > $R/gpurun_out/pmc5/sq2.log 2>&1; echo "sq2 rc=$?"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/fetch -o run -- $B > $R/gpurun_out/pmc5/fetch.log 2>&1; echo "fetch rc=$?"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/write -o run -- $B > $R/gpurun_out/pmc5/write.log 2>&1; echo "write rc=$?"
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d /tmp/tcc -o run -- $B > $R/gpurun_out/pmc5/tcc.log 2>&1; echo "tcc rc=$?"
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc5/train_pmc.md /tmp/sq1 /tmp/sq2 /tmp/fetch /tmp/write /tmp/tcc > gpurun_out/pmc5/summary.log 2>&1; echo "summary rc=$?"; find /tmp/sq1 -type f > gpurun_out/pmc5/sq1_files.txt
for f in gpurun_out/pmc5/*.log; do tail -c 20000 $f > $f.t && mv $f.t $f; done
du -sh gpurun_out
