#!/bin/bash
# GSO split on raw buffer ops: parity (GSO + encap suites) then a same-box
# A/B against a library built from another revision.
# usage: tools/sessions/gpu_gso_buf.sh TAG <libA (old)> [rounds]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; OLD=$2; R=${3:-3}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gso.py tests/test_gpu_encap.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 900 bash tools/ab_builds.sh "$OUT/ab.jsonl" "$R" "$OLD" wireglider_amd/lib/libwireglider_amd.so config3 config3udp encap
