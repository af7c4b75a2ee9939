#!/bin/bash
# One GPU-box session: build, GPU tests, smoke, bench, rocprofv3 stats.
# Stops at the first step that faults / aborts / times out (exit 124, 134,
# 137, 139 or signal); plain test failures (exit 1) do not stop the session.
# Usage: tools/gpu_session.sh [steps...]   steps: build tests alltests smoke serial serialworst serialprof kbench scan engines bench prof
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
      (cd /tmp && run serialprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/sprof" -o run -- \
         python "$ROOT/tools/bench_serial.py" --batches 30 --modes exact)
      find "$OUT/sprof" -name "*stats*" | head -20 ;;
    kbench) run kbench 300 python tools/bench_train_kernel.py ;;
    scan) run scan 300 python tools/bench_scan.py ;;
    engines) run engines 900 python tools/bench_engines.py ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
    prof)
      rm -rf "$OUT/prof"
      (cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
         python "$ROOT/bench.py" --steps 5 --warmup 2 --latency-iters 20)
      find "$OUT/prof" -name "*stats*" | head -20 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
