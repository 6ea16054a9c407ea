#!/bin/bash
# Round 4 AEAD: encrypt's partial last blocks on the whole-block path (masked)
# — parity tests (aead, encap), then alternating-process A/B against the
# previous aead.hip (tools/exp/variant_base), then the aead bench line and the
# kernel's SQ counters, then the max-ilp build A/B.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py tests/test_gpu_hostpath.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_aead.txt" 2>&1 || { tail -30 "$OUT/pytest_aead.txt"; exit 1; }
tail -1 "$OUT/pytest_aead.txt"
timeout -k 10 900 bash tools/ab_builds.sh "$OUT/ab_tail.jsonl" 3 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_base/libwireglider_amd.so aead encap > "$OUT/ab_tail.txt" 2>&1 || { tail "$OUT/ab_tail.txt"; tail "$OUT/ab_tail.jsonl.err"; exit 1; }
cat "$OUT/ab_tail.txt"
timeout -k 10 300 python3 bench.py --workload aead --steps 10 --no-cpu-baseline --no-strong --no-post > "$OUT/bench_aead.json" 2> "$OUT/bench_aead.err" || { tail -20 "$OUT/bench_aead.err"; exit 1; }
tail -1 "$OUT/bench_aead.json"
timeout -k 10 400 bash tools/counters.sh "$OUT/sq" aead aead_kernel \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
  "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LEVEL_WAVES SQ_INSTS_BRANCH" \
  "GRBM_GUI_ACTIVE GRBM_COUNT" > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
timeout -k 10 900 bash tools/ab_builds.sh "$OUT/ab_ilp.jsonl" 2 wireglider_amd/lib/libwireglider_amd.so \
  tools/exp/variant_ilp/libwireglider_amd.so aead > "$OUT/ab_ilp.txt" 2>&1 || { tail "$OUT/ab_ilp.txt"; tail "$OUT/ab_ilp.jsonl.err"; exit 1; }
cat "$OUT/ab_ilp.txt"
echo "session $TAG done"
