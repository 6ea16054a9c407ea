#!/bin/bash
# Round 6: the first-call verify kernel under rocprofv3 on the final tree
# (lane realignment in), then smoke and the default bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
O=$ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fc -o fc -- python3 tools/verify_first_call.py > $O/first_call.json 2>$O/first_call.err || { tail $O/first_call.err; exit 1; }
cut -c1-400 $O/first_call.json
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -20 "$O/smoke.txt"; exit 1; }
tail -1 "$O/smoke.txt"
timeout -k 10 600 python3 -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail "$O/bench_default.err"; exit 1; }
cut -c1-300 "$O/bench_default.json"
echo "session $TAG done"
