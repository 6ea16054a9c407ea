#!/bin/bash
# Round 4: the split kernel's loads in flight per lane (l4_unroll 8 = 94
# VGPRs / 5 waves per SIMD, 4 = 74 / 6) on the 64-B sub-batch and the mixes.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
bash tools/gpu_r03.sh "$1" ab:config4small:l4_unroll=8:l4_unroll=4 ab:config4:l4_unroll=8:l4_unroll=4 \
  ab:config5:l4_unroll=8:l4_unroll=4
