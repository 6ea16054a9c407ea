#!/bin/bash
# GRO finalize: parity of both variants, then thread loads vs LDS-staged A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_gro}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gro_finalize.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py gro gro_lds=0 gro_lds=1,gro_wide=0 gro_lds=1,gro_wide=1 > $O/ab_gro.json 2>$O/ab_gro.err; rc=$?; cat $O/ab_gro.json; [ $rc -eq 0 ] || exit $rc
