#!/bin/bash
# Round 5: the CPU baseline with per-leg warm-up and the GSO written-extent
# parity, on the lines that showed wide spreads or false parity.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_r03.sh "$TAG" bench:config3:--no-strong bench:config3udp:--no-strong bench:config4small:--no-strong \
  bench:gro:--no-strong bench:config5:--no-strong || exit 1
echo "session $TAG done"
