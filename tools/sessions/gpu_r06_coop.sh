#!/bin/bash
# Round 6: cooperative small-packet chunk loads (knob lane_coop 1 / 2) —
# parity of both variants first (lane, L4, verify and MT suites), then the
# in-process A/B on the small-packet and long-packet workloads.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
O=$ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for C in 1 2; do
  WG_LANE_COOP=$C timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lane_alignment.py tests/test_gpu_l4.py \
    tests/test_verify_gates.py tests/test_mt_batch.py tests/test_gpu_golden_l4.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > $O/pytest_coop$C.txt 2>&1 || { tail -30 $O/pytest_coop$C.txt; exit 1; }
  echo "lane_coop=$C parity: $(tail -1 $O/pytest_coop$C.txt)"
done
for W in config4small verify64d verify64 config4 config5 verify; do
  timeout -k 10 300 python3 tools/ab.py $W lane_coop=0 lane_coop=1 lane_coop=2 > $O/ab_$W.json 2> $O/ab_$W.err || { tail $O/ab_$W.err; exit 1; }
  cat $O/ab_$W.json
done
echo "session $TAG done"
