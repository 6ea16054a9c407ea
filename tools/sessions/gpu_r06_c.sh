#!/bin/bash
# Round 6: the consecutive walking kernel (verify first calls and all-small
# batches) — 8 waves per SIMD (WG_WALK8) and/or a descriptor touch for the
# grid's second half (WG_WALK_PF) against the library: each library's verify
# parity suite, the 64-B verify line (5 alternating rounds), then the first
# call on fresh streams under rocprofv3 for each library.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS="$PWD/wireglider_amd/lib/libwireglider_amd.so tools/exp/variant_walk8/libwireglider_amd.so tools/exp/variant_walk8pf/libwireglider_amd.so tools/exp/variant_walkpf/libwireglider_amd.so"
AB_PARITY_TESTS="tests/test_verify_gates.py tests/test_mt_batch.py" timeout -k 10 1000 bash tools/ab_libs.sh \
  "$OUT/ab_walk.jsonl" 5 verify64d $LIBS > "$OUT/ab_walk.txt" 2>&1; rc=$?
cat "$OUT/ab_walk.txt"; grep parity "$OUT/ab_walk.jsonl" | cut -c1-200
[ $rc -eq 0 ] || exit $rc
for L in $LIBS; do
  n=$(basename "$(dirname "$L")")
  WG_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/fc_$n" -o fc --output-format csv -- \
    python3 tools/verify_first_call.py > "$OUT/fc_$n.json" 2> "$OUT/fc_$n.err" || { tail "$OUT/fc_$n.err"; exit 1; }
  echo "first call $n done"
done
