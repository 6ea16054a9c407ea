#!/bin/bash
# Round 6: branch-free lane realignment (WG_LANE_BARREL) against the library:
# parity (L4, golden, verify, MT suites) per library, then 3 alternating
# rounds on the lane-path workloads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
AB_PARITY_TESTS="tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_verify_gates.py tests/test_mt_batch.py" \
  timeout -k 10 1100 bash tools/ab_libs.sh "$OUT/ab_barrel.jsonl" 3 config4small,verify64,verify64d,config4 \
  tools/exp/variant_barrel/libwireglider_amd.so "$PWD/wireglider_amd/lib/libwireglider_amd.so" > "$OUT/ab_barrel.txt" 2>&1; rc=$?
cat "$OUT/ab_barrel.txt"; grep parity "$OUT/ab_barrel.jsonl" | cut -c1-250
exit $rc
