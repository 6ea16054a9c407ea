#!/bin/bash
# Round 5: is the config 2 kernel slower with a process group?  The same
# bench line plain, under torch.distributed.run with no group, with a gloo
# group and with an RCCL group (one rank), then the RCCL one under a kernel
# trace.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
A="--steps 50 --no-cpu-baseline --no-strong --no-post"
run() {  # name, env..., command...
  local n=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print(sys.argv[2], d['distributed']['backend'], r['kernel_ms_avg'], r['kernel_ms_isolated'], r['frac'])" "$OUT/$n.json" "$n"
}
port() { python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])"; }
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1"
run plain X=1 python3 bench.py $A
run tr_nogroup X=1 $TR --master-port=$(port) bench.py --gpus 1 $A
run tr_gloo WG_DIST_BACKEND=gloo $TR --master-port=$(port) bench.py --gpus 1 --force-dist $A
run tr_nccl WG_DIST_BACKEND=nccl $TR --master-port=$(port) bench.py --gpus 1 --force-dist $A
run plain2 X=1 python3 bench.py $A
run nccl_direct WG_DIST_BACKEND=nccl python3 bench.py --gpus 1 --force-dist $A
run tr_nccl2 WG_DIST_BACKEND=nccl $TR --master-port=$(port) bench.py --gpus 1 --force-dist $A
(cd /tmp && WG_DIST_BACKEND=nccl timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_nccl" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 1 --force-dist $A > "$OUT/trace_nccl.json" 2> "$OUT/trace_nccl.err") || { tail "$OUT/trace_nccl.err"; exit 1; }
find "$OUT/trace_nccl" -name "*kernel_stats.csv" -exec head -8 {} \;
echo "session $TAG done"
