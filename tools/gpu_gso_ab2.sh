#!/bin/bash
# GSO parity, then spw x groups A/B and the copy-shape experiment on the same box.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-gso_ab2}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gso.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config3 gso_groups=1 gso_groups=3 gso_groups=4 gso_groups=6 gso_groups=3,gso_spw=2 gso_groups=4,gso_spw=2 > $O/ab_gso.json 2>$O/ab_gso.err; rc=$?; cat $O/ab_gso.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/exp/gso_order 2048 > $O/gso_order.txt 2>&1; head -4 $O/gso_order.txt
