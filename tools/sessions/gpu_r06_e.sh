#!/bin/bash
# Round 6: hybrid lane realignment (scalar branch when the dword offset is
# wave-uniform, mask selects otherwise) in the library against the previous
# lane code (variant_prev): parity per library, 3 alternating rounds.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
AB_PARITY_TESTS="tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_verify_gates.py tests/test_mt_batch.py tests/test_gpu_full_size.py" \
  timeout -k 10 1100 bash tools/ab_libs.sh "$OUT/ab_hybrid.jsonl" 3 config4small,verify64,verify64d,config4,config5 \
  tools/exp/variant_prev/libwireglider_amd.so "$PWD/wireglider_amd/lib/libwireglider_amd.so" > "$OUT/ab_hybrid.txt" 2>&1; rc=$?
cat "$OUT/ab_hybrid.txt"; grep parity "$OUT/ab_hybrid.jsonl" | cut -c1-250
exit $rc
