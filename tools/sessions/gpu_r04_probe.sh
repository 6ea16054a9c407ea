#!/bin/bash
# Round 4: VALU issue rates of the candidate AEAD instructions
# (tools/exp/valu_rate.hip), the rocprofv3 counter list, the first verify call
# on fresh streams under a kernel trace (kernel durations, no host work in
# them), and the config 3 / config 3 UDP / encap lines with their same-run
# copy probes.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o "$OUT/valu_rate" tools/exp/valu_rate.hip 2> "$OUT/valu_build.log" || { tail "$OUT/valu_build.log"; exit 1; }
timeout -k 10 120 "$OUT/valu_rate" > "$OUT/valu_rate.jsonl" 2>&1 || { tail "$OUT/valu_rate.jsonl"; exit 1; }
cat "$OUT/valu_rate.jsonl"
(cd /tmp && timeout -k 10 60 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1) || echo "counter list failed"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fc" -o run -- \
  python3 "$ROOT/tools/verify_first_call.py" > "$OUT/first_call.json" 2>&1) || { tail "$OUT/first_call.json"; exit 1; }
for w in config3 config3udp encap; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail "$OUT/bench_$w.err"; exit 1; }
  tail -1 "$OUT/bench_$w.json"
done
echo "session $TAG done"
