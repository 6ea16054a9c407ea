#!/bin/bash
# Round 4 encap step: the headers-only split's launch shape (blocks per
# super-buffer, waves per block) on the new AEAD, same process, interleaved.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/ab.py encap gso_groups=3 gso_groups=1 gso_groups=2 gso_groups=4 gso_groups=6 gso_groups=3,gso_waves=8 gso_groups=2,gso_waves=8 > "$OUT/ab_shape.json" 2> "$OUT/ab_shape.err" || { tail "$OUT/ab_shape.err"; exit 1; }
cat "$OUT/ab_shape.json"
echo "session $TAG done"
