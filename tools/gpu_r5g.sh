set -o pipefail
export TMPDIR=/tmp
R=/root/repo
mkdir -p $R/gpurun_out/r5g
cd /tmp
B="python3 $R/tools/bench_topk_mq.py --quick --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --kernel-trace --output-format csv -d /tmp/tq1 -o run -- $B > $R/gpurun_out/r5g/tq1.log 2>&1; echo "tq1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH --kernel-trace --output-format csv -d /tmp/tq2 -o run -- $B > $R/gpurun_out/r5g/tq2.log 2>&1; echo "tq2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/tqf -o run -- $B > $R/gpurun_out/r5g/tqf.log 2>&1; echo "tqf rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/tqw -o run -- $B > $R/gpurun_out/r5g/tqw.log 2>&1; echo "tqw rc=$?"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d /tmp/tqt -o run -- $B > $R/gpurun_out/r5g/tqt.log 2>&1; echo "tqt rc=$?"
cd $R && python3 tools/pmc_summary.py gpurun_out/r5g/topk_pmc.md /tmp/tq1 /tmp/tq2 /tmp/tqf /tmp/tqw /tmp/tqt --match topk > gpurun_out/r5g/summary.log 2>&1; echo "summary rc=$?"
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktl -o run -- python3 $R/tools/bench_engine_records.py --engines anomaly_lof > $R/gpurun_out/r5g/ktl.log 2>&1; echo "ktl rc=$?"
i=0; for f in $(find /tmp/ktl -name "*kernel_stats*"); do i=$((i+1)); cp $f $R/gpurun_out/r5g/lof_kstats_$i.csv; done
cd $R
for f in gpurun_out/r5g/*.log; do tail -c 6000 $f > $f.t && mv $f.t $f; done
