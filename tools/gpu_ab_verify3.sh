#!/bin/bash
# verify parity (all variants), header-decode A/B, SQ counters of the lane kernel.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_verify3}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_verify_gates.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py verify verify_hdr=1 verify_hdr=2 verify_hdr=0 > $O/ab_verify.json 2>$O/ab_verify.err; rc=$?; cat $O/ab_verify.json; [ $rc -eq 0 ] || exit $rc
WG_VERIFY_HDR=2 bash tools/kernel_counters.sh $O/ctr verify verify_lane_kernel
