set -u
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/frows; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest tests/test_gro_finalize.py tests/test_verify_gates.py -m gpu -q -x > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 bench.py --workload verify --steps 50 > $O/bench_verify.json 2> $O/bench_verify.err || { tail $O/bench_verify.err; exit 1; }
cat $O/bench_verify.json
timeout -k 10 300 python3 bench.py --workload gro --steps 50 > $O/bench_gro.json 2> $O/bench_gro.err || { tail $O/bench_gro.err; exit 1; }
cat $O/bench_gro.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_verify -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload verify --steps 50 --no-cpu-baseline > $O/prof_verify.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gro -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload gro --steps 50 --no-cpu-baseline > $O/prof_gro.log 2>&1 || exit 1
echo done
