#!/bin/bash
# Round 5: the row-order GSO tile kernel — parity (test_gpu_gso.py, every
# variant incl. gso_rows) then an in-process A/B on config 3 / 3udp; the
# verify first call with the per-device pool.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_gso.py tests/test_gpu_l4.py tests/test_gpu_golden_l4.py tests/test_verify_gates.py -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gso.txt" 2>&1 || { tail -40 "$OUT/pytest_gso.txt"; exit 1; }
tail -1 "$OUT/pytest_gso.txt"
timeout -k 10 300 python3 -u tools/ab.py config3 gso_rows=0 gso_rows=1 gso_rows=1,gso_tile_waves=4 gso_rows=1,gso_tile_waves=8 gso_rows=1,gso_tile_waves=12 \
  > "$OUT/ab_config3.json" 2>&1 || { tail "$OUT/ab_config3.json"; exit 1; }
cat "$OUT/ab_config3.json"
timeout -k 10 300 python3 -u tools/ab.py config3udp gso_rows=0 gso_rows=1 > "$OUT/ab_config3udp.json" 2>&1 || { tail "$OUT/ab_config3udp.json"; exit 1; }
cat "$OUT/ab_config3udp.json"
[ -f tools/exp/variant_base/libwireglider_amd.so ] && { bash tools/gpu_r03.sh "$TAG" abuild:base:config4,config5,config4small || exit 1; }
echo "session $TAG done"
