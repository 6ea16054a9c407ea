"""BASELINE configs 4 and 5 at their FULL sizes on one MI355X, checked packet
for packet against the oracle (the GPU suite held them only as
256 K / 1 M slices), and the multi-rank bench path with two ranks on one GPU
(gloo: the launch, world-size check, shards, gather and the strong-scaling
result hash the 8-GPU run is judged by).

The oracle compares in 2 M-packet slices (descriptors rebased to the slice),
so the host holds ~3 GB at a time.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
# bench.py's config 5 (16,777,216 x 1500 B, seed 0x5EED0005) results hash,
# the same at every world size (profiles/r02_n2_gloo_rehearsal.json)
CONFIG5_HASH = 544385951604289
# bench.py's config 4 batch (4,194,304 packets, 64 / 9000 B, seed 0x5EED0004)
# results hash: the config 4 strong companion's at every world size
# (profiles/r03_n2_gloo_rehearsal.json)
CONFIG4_HASH = 288304973264214192


def _wga():
    import wireglider_amd as wga

    return wga


def _compare_in_slices(buf, desc_np, out, step=1 << 21):
    """Oracle vs GPU results over descriptor slices of `step` packets."""
    n = desc_np.size
    got = out.cpu().numpy()
    for s in range(0, n, step):
        d = desc_np[s: s + step].copy()
        lo = int(d["offset"].min())
        hi = int((d["offset"] + d["len"]).max())
        host = buf[lo:hi].cpu().numpy()
        d["offset"] -= lo
        exp = oracle.l4_desc(host, d)
        np.testing.assert_array_equal(got[s: s + step], exp, err_msg=f"slice at packet {s}")


def test_config5_full_size(gpu):
    """16,777,216 x 1500 B, v4/v6 x TCP/UDP 50/50 (25.2 GB): the bench's own
    generator (same seed, same index base), so its result hash must be the
    one the multi-GPU strong-scaling line reports at every N."""
    import torch

    from wireglider_amd import dist as wdist

    wga = _wga()
    n, seg, seed = 1 << 24, 1500, 0x5EED0005
    buf = torch.empty(n * seg, dtype=torch.uint8, device=gpu)
    wga.synth_fill(buf, seed, counter_base=0)
    desc = wga.synth_desc_stride(n, seg, seg, 1, seed, 0, device=gpu)
    wga.synth_headers(buf, desc, seed, 0)
    out = wga.calc_l4_checksum_desc(buf, desc)
    torch.cuda.synchronize()
    assert wdist.result_hash(out, 0) == CONFIG5_HASH
    d = desc.cpu().numpy().view(oracle.PKT_DESC).reshape(-1)
    _compare_in_slices(buf, d, out)
    wga.store_l4csum(buf, desc, out)
    ver = wga.calc_l4_checksum_desc(buf, desc)
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(ver.to(torch.int32)).item()) == 0
    del buf, desc, out, ver
    torch.cuda.empty_cache()


def test_config4_full_size(gpu):
    """4,194,304 IPv4/UDP packets, 64 B or 9000 B 50/50 (seed 0x5EED0004),
    packed (18.9 GB): every packet's result against the oracle, then the
    generate -> store -> verify round trip."""
    import torch

    wga = _wga()
    n, seed = 1 << 22, 0x5EED0004
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < 0.5, 64, 9000).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)])
    total = int(offs[-1] + lens[-1])
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"], d["len"], d["csum_start"], d["flags"] = offs, lens, 20, 0
    buf = torch.empty(total + 16, dtype=torch.uint8, device=gpu)
    wga.synth_fill(buf, seed)
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(gpu)
    wga.synth_headers(buf, dd, seed, 0)
    out = wga.calc_l4_checksum_desc(buf, dd)
    torch.cuda.synchronize()
    from wireglider_amd import dist as wdist

    assert wdist.result_hash(out, 0) == CONFIG4_HASH
    _compare_in_slices(buf, d, out, step=1 << 20)
    wga.store_l4csum(buf, dd, out)
    ver = wga.calc_l4_checksum_desc(buf, dd)
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(ver.to(torch.int32)).item()) == 0
    del buf, dd, out, ver
    torch.cuda.empty_cache()


def test_bench_two_ranks_on_one_gpu(gpu, tmp_path):
    """`bench.py --gpus 2` starts two ranks itself (torch.distributed.run on
    127.0.0.1), they find a 2-rank group, shard config 2 (weak) and config 5
    (strong) and config 4's bimodal batch split by bytes (strong), and rank 0
    prints one line whose whole-job numbers and result hashes are the 8-GPU
    run's logic at N = 2 (gloo: both ranks share this GPU)."""
    env = dict(os.environ)
    env["WG_DIST_BACKEND"] = "gloo"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--settle-seconds", "0.05"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["distributed"]["world_size"] == 2
    assert len(line["distributed"]["kernel_ms_per_rank"]) == 2
    assert line["post_checks"]["verify_nonzero"] == 0
    assert line["post_checks"]["gathered_results"] == 2 * (1 << 20)
    assert line["strong_scaling"]["result_hash"] == CONFIG5_HASH
    assert line["strong_scaling"]["packets_per_rank"] == [1 << 23, 1 << 23]
    # config 4's one bimodal batch split by bytes: the N = 1 hash, byte totals
    # within one 9000-B packet
    s4 = line["strong_scaling_config4"]
    assert s4["result_hash"] == CONFIG4_HASH
    assert sum(s4["packets_per_rank"]) == 1 << 22
    assert max(s4["bytes_per_rank"]) - min(s4["bytes_per_rank"]) <= 9000


def test_bench_rccl_one_rank(gpu, tmp_path):
    """The RCCL branch of the multi-GPU path, on one GPU:
    bench.py under torch.distributed.run --nproc-per-node=1 with
    --force-dist and WG_DIST_BACKEND=nccl creates the process group with
    init_process_group("nccl", device_id=...) and runs every collective the
    8-GPU run uses on device tensors — the uint8 all_gather of the results
    (gather_results), the int64 all_reduce of the hashes (allreduce_hash)
    and of the verify count, the float64 max (max_over_ranks) and all_gather
    (all_gather_floats), barriers — and still reproduces the N = 1 hashes."""
    import socket

    env = dict(os.environ)
    env["WG_DIST_BACKEND"] = "nccl"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"),
                        "--gpus", "1", "--force-dist", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--settle-seconds", "0.05"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print("rccl_one_rank", json.dumps({k: line[k] for k in ("distributed", "post_checks", "value")}))
    assert line["distributed"]["backend"] == "nccl" and line["distributed"]["world_size"] == 1
    assert line["n_gpus"] == 1 and len(line["distributed"]["kernel_ms_per_rank"]) == 1
    assert line["post_checks"]["verify_nonzero"] == 0
    assert line["post_checks"]["gathered_results"] == 1 << 20
    assert line["strong_scaling"]["result_hash"] == CONFIG5_HASH
    assert line["strong_scaling_config4"]["result_hash"] == CONFIG4_HASH
