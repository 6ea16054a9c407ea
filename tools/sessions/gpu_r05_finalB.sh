#!/bin/bash
# Round 5 evidence, part B: the other workloads' lines (CPU baselines on
# fixed CPUs per leg), then config 4 / 5 kernel statistics.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_r03.sh "$TAG" bench:config1:--no-strong bench:config4:--no-strong bench:config4small:--no-strong \
  bench:config5:--no-strong bench:verify:--no-strong bench:verify64d:--no-strong bench:gro:--no-strong \
  bench:aead:--no-strong bench:encap:--no-strong || exit 1
echo "session $TAG done"
