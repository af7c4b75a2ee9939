#!/bin/bash
# H2D-bound headline step with the rank's threads on the GPU's NUMA node
# (auto), on the other node, and unbound. One GPU; each run time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in auto 1 off auto; do
  echo "=== JB_NUMA_BIND=$mode"
  JB_NUMA_BIND=$mode timeout -k 10 240 python bench.py --steps 30 --warmup 5 \
    > gpurun_out/numa_$mode.json 2> gpurun_out/numa_$mode.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['numa_node'])" gpurun_out/numa_$mode.json
done
