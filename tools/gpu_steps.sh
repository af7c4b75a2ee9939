#!/bin/bash
# Run GPU steps in order on a gpurun box, each under its own time limit.
# A step that fails normally (a failing test) lets the next one run; a step
# ended by its time limit, an abort or a segmentation fault (124, 134, 137,
# 139) ends the call - nothing more touches the GPU after it.
#   tools/gpu_steps.sh "timeout -k 10 300 python -u -m pytest ..." "..."
mkdir -p gpurun_out
for step in "$@"; do
  bash -c "$step"
  rc=$?
  echo "[step rc=$rc] $step" >> gpurun_out/steps.log
  case $rc in
    124|134|137|139) echo "stopping after rc=$rc" >> gpurun_out/steps.log; exit $rc ;;
  esac
done
exit 0
