#!/bin/bash
# One GPU-box session: build, GPU tests, smoke, bench, rocprofv3 stats.
# Stops at the first step that faults / aborts / times out (exit 124, 134,
# 137, 139 or signal); plain test failures (exit 1) do not stop the session.
# Usage: tools/gpu_session.sh [steps...]   steps: build tests alltests smoke serial serialworst serialprof kbench scan
#        engines bench prof lof topk gaps pmc_train pmc_topk pmc_select pmc_lof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${*:-build tests smoke bench prof}

run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== [$name] $(date +%T) $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -5 "$OUT/$name.log"
  case $rc in
    0|1|2|5) return 0 ;;
    *) echo "fatal rc=$rc in $name: stopping"; exit $rc ;;
  esac
}

for s in $STEPS; do
  case $s in
    build) run build 600 python -m jubatus_amd.build_ext ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    alltests) run pytest_all 1200 python -m pytest tests -x -q ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    serial) run serial 400 python tools/bench_serial.py --batches 40 --modes exact ;;
    serialworst) run serialworst 400 python tools/bench_serial.py --batches 8 --modes exact --worst-case ;;
    serialprof)
      rm -rf "$OUT/sprof"
      (cd /tmp && run serialprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sprof" -o run -- \
         python "$ROOT/tools/bench_serial.py" --batches 30 --modes exact)
      find "$OUT/sprof" -name "*stats*" | head -20 ;;
    kbench) run kbench 300 python tools/bench_train_kernel.py ;;
    scan) run scan 300 python tools/bench_scan.py ;;
    engines) run engines 900 python tools/bench_engines.py ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
    prof)
      rm -rf "$OUT/prof"
      (cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
         python "$ROOT/bench.py" --steps 5 --warmup 2 --latency-iters 20)
      find "$OUT/prof" -name "*stats*" | head -20 ;;
    lof)   # LOF engine record (native server over RPC) + its kernel stats
      run lof 300 python tools/bench_engine_records.py --engines anomaly_lof
      rm -rf /tmp/lofprof
      (cd /tmp && run lofprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lofprof -o run -- \
         python3 "$ROOT/tools/bench_engine_records.py" --engines anomaly_lof) || exit $?
      cp /tmp/lofprof/run_kernel_stats.csv "$OUT/lof_kernel_stats.csv" ;;
    topk)  # signature / score top-k paths below 2M rows (select vs the previous default)
      run topk_100k 300 python tools/bench_topk_lsh.py --rows 100000 --iters 200 \
        --cases 1:10,4:10,1:31,4:40,1:94 --paths fused,select,default --metrics 1,0
      run topk_1m 300 python tools/bench_topk_lsh.py --rows 1000000 --iters 100 \
        --cases 1:10,4:10,1:31,4:40,1:100 --paths fused,select,default --metrics 1
      run topk_scores 300 python tools/bench_topk_scores.py --rows 1000000 --iters 100 --paths chain,fused,select,default ;;
    gaps)  # kernel-trace gaps of the exact-mode committer
      rm -rf /tmp/ktv
      (cd /tmp && run gaps_trace 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ktv -o run -- \
         python3 "$ROOT/tools/bench_serial.py" --batches 30 --modes exact) || exit $?
      python3 tools/trace_gaps.py /tmp/ktv "$OUT/gaps_steady.md" --last 1500 > /dev/null
      python3 tools/trace_gaps.py /tmp/ktv "$OUT/gaps_all.md" > /dev/null ;;
    pmc_train|pmc_topk|pmc_select|pmc_lof)   # counter passes, one rocprofv3 run each (block limits per pass)
      case $s in
        pmc_train) B="python3 $ROOT/tools/bench_serial.py --batches 6 --modes exact,atomic"; M="" ;;
        pmc_topk) B="python3 $ROOT/tools/bench_topk_mq.py --quick --iters 3"; M="--match topk" ;;
        pmc_select) B="python3 $ROOT/tools/bench_topk_lsh.py --rows 1000000 --iters 20 --cases 1:31,4:40 --paths select --metrics 1"
                    M="--match select" ;;
        *) B="python3 $ROOT/tools/bench_lof_kernel.py --batches 40"; M="--match lof" ;;
      esac
      P=0
      for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
               "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" \
               "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        P=$((P + 1)); rm -rf /tmp/pmc$P
        (cd /tmp && run ${s}_$P 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/pmc$P -o run -- $B) \
          || exit $?
      done
      python3 tools/pmc_summary.py "$OUT/$s.md" /tmp/pmc1 /tmp/pmc2 /tmp/pmc3 /tmp/pmc4 /tmp/pmc5 $M ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
