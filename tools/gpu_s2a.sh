set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/s2a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gso.py tests/test_gpu_l4.py tests/test_verify_gates.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config3 gso_groups=1 gso_groups=2 gso_groups=3 gso_groups=6 gso_groups=12 gso_groups=3,gso_waves=8 gso_groups=6,gso_waves=8 > $O/ab_gso.json 2>$O/ab_gso.err; rc=$?; cat $O/ab_gso.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config5 l4_pf=0 l4_pf=16 l4_pf=64 l4_pf=128 l4_pf=256 l4_pf=512 > $O/ab_c5.json 2>$O/ab_c5.err; rc=$?; cat $O/ab_c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py verify l4_pf=0 > $O/ab_verify.json 2>$O/ab_verify.err; rc=$?; cat $O/ab_verify.json; [ $rc -eq 0 ] || exit $rc
