#!/bin/bash
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
port() { python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])"; }
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1"
timeout -k 10 200 python3 tools/dist_hiccup_probe.py --nogroup > "$OUT/nogroup.json" 2> "$OUT/nogroup.err" || { tail "$OUT/nogroup.err"; exit 1; }
cat "$OUT/nogroup.json"
WG_DIST_BACKEND=nccl timeout -k 10 200 $TR --master-port=$(port) tools/dist_hiccup_probe.py > "$OUT/nccl.json" 2> "$OUT/nccl.err" || { tail "$OUT/nccl.err"; exit 1; }
grep '^{' "$OUT/nccl.json"
WG_DIST_BACKEND=nccl TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 timeout -k 10 200 $TR --master-port=$(port) tools/dist_hiccup_probe.py > "$OUT/nccl_nomon.json" 2> "$OUT/nccl_nomon.err" || { tail "$OUT/nccl_nomon.err"; exit 1; }
grep '^{' "$OUT/nccl_nomon.json"
echo "session $TAG done"
