#!/bin/bash
# Verify-gates kernel: parity of every variant, then descriptor mode x occupancy A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_verify}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_verify_gates.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py verify verify_dm=0 verify_dm=0,verify_occ=0 verify_dm=2,verify_occ=6 verify_dm=2,verify_occ=0 verify_dm=2,verify_occ=6,l4_iters=8 > $O/ab_verify.json 2>$O/ab_verify.err; rc=$?; cat $O/ab_verify.json; [ $rc -eq 0 ] || exit $rc
