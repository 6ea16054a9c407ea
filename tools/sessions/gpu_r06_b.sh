#!/bin/bash
# Round 6: walking-kernel descriptor prefetch (WG_WALK_PF) A/B on the 64-B
# verify line, with each library's verify parity suite first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
AB_PARITY_TESTS="tests/test_verify_gates.py tests/test_mt_batch.py" timeout -k 10 1000 bash tools/ab_libs.sh \
  "$OUT/ab_walkpf.jsonl" 5 verify64d tools/exp/variant_walkpf/libwireglider_amd.so \
  "$PWD/wireglider_amd/lib/libwireglider_amd.so" > "$OUT/ab_walkpf.txt" 2>&1; rc=$?
cat "$OUT/ab_walkpf.txt"; grep parity "$OUT/ab_walkpf.jsonl" | cut -c1-300
exit $rc
