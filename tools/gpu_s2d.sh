set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/s2d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gso.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab.py config3 gso_spw=0 gso_spw=1 gso_spw=2 gso_groups=2 gso_groups=3 gso_groups=6 gso_groups=12 gso_spw=2,gso_groups=3 > $O/ab_gso.json 2>$O/ab_gso.err; rc=$?; cat $O/ab_gso.json; [ $rc -eq 0 ] || exit $rc
