#!/bin/bash
# GSO parity (every variant) + config3 bench + rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-gso_check}; mkdir -p $O
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gso.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload config3 --steps 30 > $O/bench_config3.json 2> $O/bench_config3.err || { tail $O/bench_config3.err; exit 1; }
cat $O/bench_config3.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats_config3" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload config3 --steps 30 --no-cpu-baseline > "$O/stats_config3.log" 2>&1) || { echo "stats failed"; tail "$O/stats_config3.log"; exit 1; }
grep -E "gso_" $O/stats_config3/run_kernel_stats.csv | cut -c1-140
