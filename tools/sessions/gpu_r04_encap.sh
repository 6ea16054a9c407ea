#!/bin/bash
# Round 4 encap step: pipelined slices (encap_parts: the headers-only split of
# slice k on a side stream under slice k-1's AEAD) and the split's segments
# per wave step (encap_spw), same process, interleaved, on the new AEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/ab.py encap encap_parts=1 encap_parts=2 encap_parts=3 encap_parts=4 encap_parts=8 > "$OUT/ab_parts.json" 2> "$OUT/ab_parts.err" || { tail "$OUT/ab_parts.err"; exit 1; }
cat "$OUT/ab_parts.json"
timeout -k 10 400 python3 -u tools/ab.py encap encap_spw=2 encap_spw=3 encap_spw=4 encap_spw=0 > "$OUT/ab_spw.json" 2> "$OUT/ab_spw.err" || { tail "$OUT/ab_spw.err"; exit 1; }
cat "$OUT/ab_spw.json"
echo "session $TAG done"
