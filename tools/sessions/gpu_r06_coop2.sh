#!/bin/bash
# Round 6: lane_coop back to back (bench.py lines, alternating processes):
# config 4's 64-B sub-batch 0 / 1, uniform 64-B verify 0 / 2.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
O=$ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for spec in config4small:0 config4small:1 verify64:0 verify64:2; do
    W=${spec%%:*}; C=${spec##*:}
    WG_LANE_COOP=$C timeout -k 10 200 python3 bench.py --workload $W --no-cpu-baseline --no-post --steps 200 > $O/b_${W}_${C}_$r.json 2> $O/b_${W}_${C}_$r.err || { tail $O/b_${W}_${C}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_${W}_${C}_$r.json').read().strip().splitlines()[-1]); print('$W', 'lane_coop=$C', 'round $r', d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
  done
done
echo "session $TAG done"
