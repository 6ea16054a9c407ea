#!/bin/bash
# GRO bench + stats, and a 2-rank rehearsal of the multi-GPU bench path on one
# GPU (gloo backend: both ranks share cuda:0; the 8-GPU RCCL run is the driver's).
set -u
cd "${GRAFT_REPO_ROOT}"
O=$(pwd)/gpurun_out/${1:-gro_dist}; mkdir -p $O
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload gro --steps 100 > $O/bench_gro.json 2> $O/bench_gro.err || { tail $O/bench_gro.err; exit 1; }
cat $O/bench_gro.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats_gro" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload gro --steps 100 --no-cpu-baseline > "$O/stats_gro.log" 2>&1) || { echo "stats gro failed"; tail "$O/stats_gro.log"; exit 1; }
WG_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_2rank.json 2> $O/bench_2rank.err || { tail $O/bench_2rank.err; exit 1; }
cat $O/bench_2rank.json
echo done
