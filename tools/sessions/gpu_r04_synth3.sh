#!/bin/bash
# Round 4 encap synthesis, second form (fast prologue loads, v_sad_u16 sums,
# the checksum weight parked in LDS, the split walking a list of the
# super-buffers left to it): parity, A/B encap_synth 0 / 1, kernel statistics
# and SQ counters of the synthesizing AEAD.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encap.py tests/test_gpu_aead.py tests/test_gpu_gso.py tests/test_gpu_hostpath.py \
  tests/test_verify_gates.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 400 python3 -u tools/ab.py encap encap_synth=0 encap_synth=1 > "$OUT/ab_synth.json" 2> "$OUT/ab_synth.err" || { tail "$OUT/ab_synth.err"; exit 1; }
cat "$OUT/ab_synth.json"
(cd /tmp && WG_ENCAP_SYNTH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_synth1" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --workload encap --steps 10 --no-cpu-baseline --no-strong --no-post > "$OUT/stats_synth1.log" 2>&1) || { echo "stats failed"; tail "$OUT/stats_synth1.log"; exit 1; }
WG_ENCAP_SYNTH=1 timeout -k 10 400 bash tools/counters.sh "$OUT/sq1" encap aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" > "$OUT/sq1.log" 2>&1 || { tail -20 "$OUT/sq1.log"; exit 1; }
cat "$OUT/sq1/summary.json"
echo "session $TAG done"
