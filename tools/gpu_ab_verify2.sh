#!/bin/bash
# Whole -m gpu suite, then the verify kernel's header source A/B (byte gather
# lanes vs a separate header load) x occupancy, interleaved in one process.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_verify2}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py verify verify_hdr=0 verify_hdr=1 verify_hdr=1,verify_occ=0 verify_hdr=0,verify_occ=0 > $O/ab_verify.json 2>$O/ab_verify.err; rc=$?; cat $O/ab_verify.json; [ $rc -eq 0 ] || exit $rc
