#!/bin/bash
# Descriptor-mode A/B for the descriptor-batch L4 kernel (tools/ab.py) after
# the parity tests of every variant.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_desc}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_l4.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config5 l4_descv=0 l4_descv=1 l4_descv=2 l4_descv=2,l4_occ=0 l4_descv=2,l4_iters=4 l4_descv=2,l4_iters=8 l4_descv=2,l4_iters=4,l4_occ=0 > $O/ab_c5.json 2>$O/ab_c5.err; rc=$?; cat $O/ab_c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config4 l4_descv=0 l4_descv=2 l4_descv=2,l4_occ=0 l4_descv=2,l4_iters=4 > $O/ab_c4.json 2>$O/ab_c4.err; rc=$?; cat $O/ab_c4.json; [ $rc -eq 0 ] || exit $rc
