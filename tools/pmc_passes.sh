set -e
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_engines.py -k "topk or pool or sparse" > gpurun_out/pmc/tests.log 2>&1
timeout -k 10 200 python -u tools/pmc_engines.py > gpurun_out/pmc/eng_time.jsonl 2>&1
JB_TOPK_WQ_OFF=1 timeout -k 10 200 python -u tools/pmc_engines.py > gpurun_out/pmc/eng_time_wqoff.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/pmc_engines.py --iters 5"
B="python3 bench.py --steps 3 --warmup 1 --no-rpc --batches-per-step 4 --warmup-pools 2 --latency-iters 5"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/e_fetch -o run -- $P > gpurun_out/pmc/e1.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/e_write -o run -- $P > gpurun_out/pmc/e2.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/e_sq -o run -- $P > gpurun_out/pmc/e3.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc/e_tcc -o run -- $P > gpurun_out/pmc/e4.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/t_write -o run -- $B > gpurun_out/pmc/t2.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/t_sq -o run -- $B > gpurun_out/pmc/t3.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc/t_tcc -o run -- $B > gpurun_out/pmc/t4.log 2>&1
echo done
