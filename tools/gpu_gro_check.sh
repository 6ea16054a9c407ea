#!/bin/bash
# GRO finalize parity (every variant), bench line, and the variants A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-gro_check}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gro_finalize.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload gro --steps 30 > $O/bench_gro.json 2> $O/bench_gro.err || { tail $O/bench_gro.err; exit 1; }
cat $O/bench_gro.json
timeout -k 10 300 python3 -u tools/ab.py gro gro_chunks=5 gro_chunks=4 gro_lds=1,gro_wide=0 gro_lds=0 > $O/ab_gro.json 2>$O/ab_gro.err; rc=$?; cat $O/ab_gro.json; [ $rc -eq 0 ] || exit $rc
