#!/bin/bash
# L4 kernel occupancy A/B (tools/ab.py) after the parity tests of every variant.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_occ}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_l4.py tests/test_verify_gates.py tests/test_gpu_gso.py tests/test_gpu_dropin.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for W in config2 config5 config4; do
  timeout -k 10 300 python3 -u tools/ab.py $W l4_occ=0 l4_occ=7 l4_occ=8 > $O/ab_$W.json 2>$O/ab_$W.err; rc=$?; cat $O/ab_$W.json; [ $rc -eq 0 ] || exit $rc
done
