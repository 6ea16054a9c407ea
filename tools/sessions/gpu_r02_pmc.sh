#!/bin/bash
# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) + kernel stats for
# the given workloads; summaries land in gpurun_out/r02_pmc/<w>/pmc_<w>.json.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
export TMPDIR=/tmp
for w in "$@"; do
  OUT=$ROOT/gpurun_out/r02_pmc/$w
  mkdir -p $OUT
  bash tools/pmc_profile.sh $OUT --workload $w --steps 10 --settle-seconds 0.1 --no-strong > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/pmc_$w.json')); print('$w', d.get('hbm_bytes_per_launch'))"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
     python3 $ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-strong --workload $w > $OUT/prof.json 2> $OUT/prof.err)
  find $OUT/prof -name "*kernel_stats.csv" -exec head -3 {} \;
done
