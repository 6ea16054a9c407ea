#!/bin/bash
# Round 5, first session: smoke, the whole GPU suite (incl. the RCCL
# one-rank bench test), the verify first call under a kernel trace, the
# drop-in at 1 and 16 threads, and the config 2 line.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/gpu_r03.sh "$TAG" tests || exit 1
timeout -k 10 200 python3 -u tools/verify_first_call.py > "$OUT/first_call.json" 2> "$OUT/first_call.err" || { tail "$OUT/first_call.err"; exit 1; }
cut -c1-600 "$OUT/first_call.json"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/first_call_trace" -o run -- \
  python3 -u "$ROOT/tools/verify_first_call.py" > "$OUT/first_call_traced.json" 2> "$OUT/first_call_traced.err") || { tail "$OUT/first_call_traced.err"; exit 1; }
g++ -std=c++20 -O2 -I include tests/cpp/percall_latency.cpp -L wireglider_amd/lib -lwireglider_amd \
  -Wl,-rpath,"$ROOT/wireglider_amd/lib" -lpthread -o "$OUT/percall_latency" || exit 1
timeout -k 10 120 env -u WG_PERCALL "$OUT/percall_latency" 200000 1 16 > "$OUT/percall_threads.json" || exit 1
cat "$OUT/percall_threads.json"
bash tools/gpu_r03.sh "$TAG" bench:config2 || exit 1
echo "session $TAG done"
