#!/bin/bash
# One GPU-box session: parity tests, smoke, bench line, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/fault/timeout ends the script.
# usage: tools/sessions/gpu_check.sh [tag] [pytest-args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
TAG=${1:-r01}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_if_fatal() {  # $1 = exit code, $2 = step name
  case "$1" in
    0) return 0 ;;
    1) echo "[$2] failures (exit 1), continuing"; return 0 ;;
    *) echo "[$2] fatal exit $1 -> stopping"; exit "$1" ;;
  esac
}

echo "== build check"; python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 3; }
echo "== pytest -m gpu"
timeout -k 10 900 python3 -m pytest tests -m gpu -q -x ${@:2} > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -5 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest
echo "== smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
tail -2 "$OUT/smoke.log"; stop_if_fatal $rc smoke
echo "== bench"
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; stop_if_fatal $rc bench
echo "== rocprofv3 kernel stats"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1; rc=$?
tail -3 "$OUT/prof.log"; stop_if_fatal $rc rocprof
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | head -20
echo done
