#!/bin/bash
# New long-packet parity test + config3 bench with its whole-output post-check.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-c3post}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_l4.py -m gpu -k long > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload config3 --steps 30 > $O/bench_config3.json 2> $O/bench_config3.err || { tail $O/bench_config3.err; exit 1; }
cat $O/bench_config3.json
