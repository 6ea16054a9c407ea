#!/bin/bash
# Round-2 bench session on one GPU box: GPU tests, the default bench line
# (config 2 + config 5 strong-scaling companion), config 1 and the UDP_L4
# GSO variant, and a 2-rank rehearsal of the self-spawning multi-rank path
# (gloo, both ranks on the one GPU).  Every GPU step has its own time limit;
# the first failure ends the script.
# usage: tools/sessions/gpu_r02_bench.sh TAG [workloads...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-r02}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import os, json; print(json.dumps({'affinity': len(os.sched_getaffinity(0)), 'cpu_count': os.cpu_count()}))" > "$OUT/host_cores.json"  # bench.py's cpu_baseline reports the granted cores
cat /sys/fs/cgroup/cpu.max >> "$OUT/host_cores.json" 2>/dev/null || true
nproc >> "$OUT/host_cores.json"
echo "== pytest -m gpu"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
grep -h "percall_latency" "$OUT/pytest_gpu.log" > "$OUT/percall_latency.txt" || true
echo "== bench default"
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err"
cat "$OUT/bench_config2.json"
for w in "$@"; do
  echo "== bench $w"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --no-strong --workload "$w" > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  cat "$OUT/bench_$w.json"
done
echo "== 2-rank rehearsal (gloo, one GPU)"
WG_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
  > "$OUT/bench_n2_gloo.json" 2> "$OUT/bench_n2_gloo.err"
cat "$OUT/bench_n2_gloo.json"
echo done
