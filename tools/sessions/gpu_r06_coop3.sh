#!/bin/bash
# Round 6: the final lane_coop build (split kernel's lane role only, default
# 1) — parity with the default and with lane_coop 0, then back-to-back lines
# alternating 0 / 1 on config 4's 64-B sub-batch and config 4.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
O=$ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for C in 1 0; do
  WG_LANE_COOP=$C timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lane_alignment.py tests/test_gpu_l4.py \
    tests/test_gpu_golden_l4.py tests/test_gpu_full_size.py tests/test_mt_batch.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > $O/pytest_coop$C.txt 2>&1 || { tail -30 $O/pytest_coop$C.txt; exit 1; }
  echo "lane_coop=$C parity: $(tail -1 $O/pytest_coop$C.txt)"
done
for r in 1 2 3; do
  for spec in config4small:0 config4small:1 config4:0 config4:1; do
    W=${spec%%:*}; C=${spec##*:}
    WG_LANE_COOP=$C timeout -k 10 200 python3 bench.py --workload $W --no-cpu-baseline --no-post > $O/b_${W}_${C}_$r.json 2> $O/b_${W}_${C}_$r.err || { tail $O/b_${W}_${C}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_${W}_${C}_$r.json').read().strip().splitlines()[-1]); print('$W', 'lane_coop=$C', 'round $r', d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
  done
done
echo "session $TAG done"
