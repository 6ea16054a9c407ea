#!/bin/bash
# Round 5 evidence, part A: smoke, the whole GPU suite, config 2 (PMC + line +
# kernel statistics), config 3 UDP_L4 (PMC + line + statistics), config 3
# line, the RCCL one-rank line, encap PMC with header synthesis off.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$ROOT"
TAG=$1
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/gpu_r03.sh "$TAG" tests evidence:config2 evidence:config3udp:--no-strong bench:config3:--no-strong || exit 1
port=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
WG_DIST_BACKEND=nccl timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
  --master-addr 127.0.0.1 --master-port=$port bench.py --gpus 1 --force-dist --steps 20 --no-cpu-baseline \
  > "$OUT/rccl_one_rank.json" 2> "$OUT/rccl_one_rank.err" || { tail "$OUT/rccl_one_rank.err"; exit 1; }
cut -c1-300 "$OUT/rccl_one_rank.json"
WG_ENCAP_SYNTH=0 bash tools/pmc_profile.sh "$OUT/pmc_encap_nosynth" --workload encap --steps 10 --settle-seconds 0.1 --no-strong \
  > "$OUT/pmc_encap_nosynth.log" 2>&1 || { tail "$OUT/pmc_encap_nosynth.log"; exit 1; }
echo "session $TAG done"
