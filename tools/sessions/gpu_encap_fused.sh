#!/bin/bash
# The fused encap step (wg_encap_batch): parity tests, the fused and two-call
# bench lines on one box, and a kernel-trace profile of the fused one.
# usage: tools/sessions/gpu_encap_fused.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_encap.py tests/test_gpu_gso.py tests/test_capi.py > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
for w in encap encap_2call encap; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"
  python3 -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], d['post_checks'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 \
  --workload encap --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -12
