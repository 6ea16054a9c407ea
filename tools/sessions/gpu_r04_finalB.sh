#!/bin/bash
# Round 4 final evidence, part B: the other bench lines on one box.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
bash tools/gpu_r03.sh "$1" bench:config1 bench:config3 bench:config3udp bench:config4 bench:config4small \
  bench:config5 bench:verify bench:verify64d bench:gro
