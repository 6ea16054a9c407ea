#!/bin/bash
# Round 4 encap: header synthesis in the AEAD (encap_synth) — encap / AEAD /
# GSO / host-path parity, the interleaved A/B of encap_synth 0 / 1 on the
# encap workload, K = 4 blocks per lane on the AEAD / encap workloads, then
# the pending L4 lane-role rotation session.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encap.py tests/test_gpu_aead.py tests/test_gpu_hostpath.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest_encap.txt" 2>&1 || { tail -40 "$OUT/pytest_encap.txt"; exit 1; }
tail -1 "$OUT/pytest_encap.txt"
timeout -k 10 400 python3 -u tools/ab.py encap encap_synth=0 encap_synth=1 > "$OUT/ab_synth.json" 2> "$OUT/ab_synth.err" || { tail "$OUT/ab_synth.err"; exit 1; }
cat "$OUT/ab_synth.json"
timeout -k 10 400 python3 -u tools/ab.py aead aead_k=0 aead_k=4 > "$OUT/ab_k4_aead.json" 2> "$OUT/ab_k4_aead.err" || { tail "$OUT/ab_k4_aead.err"; exit 1; }
cat "$OUT/ab_k4_aead.json"
timeout -k 10 400 python3 -u tools/ab.py encap aead_k=0 aead_k=4 encap_synth=1 encap_synth=1,aead_k=4 > "$OUT/ab_k4_encap.json" 2> "$OUT/ab_k4_encap.err" || { tail "$OUT/ab_k4_encap.err"; exit 1; }
cat "$OUT/ab_k4_encap.json"
bash tools/sessions/gpu_r04_rot.sh "$TAG/rot"
