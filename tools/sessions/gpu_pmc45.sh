#!/bin/bash
# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE passes) for configs 4 and 5.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-pmc45}; mkdir -p $O
for W in config5 config4; do
  bash tools/pmc_profile.sh "$O/pmc_$W" --workload $W --steps 10 --settle-seconds 0.1 > "$O/pmc_$W.log" 2>&1 || { tail "$O/pmc_$W.log"; exit 1; }
  tail -4 "$O/pmc_$W.log"
done
