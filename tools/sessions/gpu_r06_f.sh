#!/bin/bash
# Round 6: the final lane realignment (hybrid on descriptor batches, the
# per-word select on uniform batches) against variant_prev, then the whole
# GPU suite on the library.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
AB_PARITY_TESTS="tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_verify_gates.py" \
  timeout -k 10 900 bash tools/ab_libs.sh "$OUT/ab_lane.jsonl" 3 config4small,verify64,verify64d,config4 \
  tools/exp/variant_prev/libwireglider_amd.so "$PWD/wireglider_amd/lib/libwireglider_amd.so" > "$OUT/ab_lane.txt" 2>&1; rc=$?
cat "$OUT/ab_lane.txt"; grep parity "$OUT/ab_lane.jsonl" | cut -c1-200
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03.sh "$1" tests
