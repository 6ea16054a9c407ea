#!/bin/bash
# Interleaved A/B (tools/ab.py) of knob variants on workloads.
# usage: tools/sessions/gpu_r02_ab.sh TAG "workload variants..." ["workload variants..."]
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for spec in "$@"; do
  w=${spec%% *}
  timeout -k 10 300 python3 tools/ab.py $spec > $OUT/ab_$w.json
  cat $OUT/ab_$w.json
done
