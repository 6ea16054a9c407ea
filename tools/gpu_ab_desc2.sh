#!/bin/bash
# Descriptor-mode A/B, second pass: vector descriptor loads x occupancy.
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-ab_desc2}; mkdir -p $O
for W in config5 config4; do
  timeout -k 10 300 python3 -u tools/ab.py $W l4_descv=0 l4_descv=1 l4_descv=1,l4_occ=0 l4_descv=1,l4_occ=8 l4_descv=2,l4_iters=4,l4_occ=0 > $O/ab_$W.json 2>$O/ab_$W.err; rc=$?; cat $O/ab_$W.json; [ $rc -eq 0 ] || exit $rc
done
