#!/bin/bash
# GSO parity (every variant), then block size (waves per block) x groups A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-gso_ab3}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gso.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/ab.py config3 gso_groups=3,gso_waves=4 gso_groups=12,gso_waves=1 gso_groups=6,gso_waves=2 gso_groups=16,gso_waves=1 gso_groups=8,gso_waves=1 gso_groups=23,gso_waves=1 gso_groups=12,gso_waves=1,gso_spw=2 > $O/ab_gso.json 2>$O/ab_gso.err; rc=$?; cat $O/ab_gso.json; [ $rc -eq 0 ] || exit $rc
