"""World-size-2 (and 3) gloo tests of the sharded path on CPU.

The sharding, result gather and hash reduction are the same code the GPU
bench runs over RCCL; here each rank's per-shard compute is the CPU oracle
(test infrastructure), so the test checks that the sharded job reproduces
the single-process answer bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wireglider_amd import dist as wdist


BIG_OFFSET = (1 << 39) + 12345


def exact_hash(values, offset: int) -> int:
    """The hash's definition in Python integers (no overflow possible)."""
    return sum((offset + 1 + i) * (int(x) + 1) for i, x in enumerate(values)) % wdist.HASH_MOD


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_batch(n, seed=5):
    """Deterministic variable-length batch: (bytes, desc structured array)."""
    import oracle

    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < 0.5, 64, rng.integers(40, 3000, n)).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)])
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"], d["len"] = offs, lens
    d["flags"] = rng.integers(0, 4, n)
    d["csum_start"] = np.where(d["flags"] & 1, 40, 20)
    return buf, d


def _worker(rank, world, port, n, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "oracle"), str(root / "tests")]
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        buf, d = make_batch(n)
        bounds = wdist.shard_bounds_by_bytes(d["len"], world)
        lo, hi = bounds[rank]
        local = torch.from_numpy(oracle.l4_desc(buf, d[lo:hi], threads=1).astype(np.int32)).to(torch.uint16)
        sent = []
        real = dist.all_gather

        def spy(parts, t, group=None):
            sent.append((str(t.dtype), t.numel() * t.element_size()))
            return real(parts, t, group=group)

        dist.all_gather = spy
        try:
            full = wdist.gather_results(local, [b - a for a, b in bounds])
        finally:
            dist.all_gather = real
        h = wdist.allreduce_hash(wdist.result_hash(local, lo))
        # far from zero: per-rank hashes near 2^61 must not overflow the reduction
        h_big = wdist.allreduce_hash(wdist.result_hash(local, lo + BIG_OFFSET))
        t = wdist.max_over_ranks(float(rank + 1))
        per = wdist.all_gather_floats([float(rank), 0.5 * rank])
        if rank == 0:
            q.put((full.numpy().astype(np.uint16).tobytes(), h, h_big, t, bounds, per, sent))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_sharded_equals_single_process(world):
    import oracle

    n = 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    full_bytes, h, h_big, t, bounds, per, sent = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, d = make_batch(n)
    ref = oracle.l4_desc(buf, d)
    got = np.frombuffer(full_bytes, dtype=np.uint16)
    np.testing.assert_array_equal(got, ref)
    assert h == wdist.result_hash(torch.from_numpy(ref.astype(np.int32)), 0) == exact_hash(ref, 0)
    assert h_big == exact_hash(ref, BIG_OFFSET)
    assert t == float(world)
    assert per == [[float(r), 0.5 * r] for r in range(world)]  # per-rank bench times, in rank order
    # the gather moves 2 B per packet of the longest shard
    assert sent == [("torch.uint8", 2 * max(b - a for a, b in bounds))]
    # byte balance: each shard within one max-size packet of the mean
    per = [int(d["len"][a:b].astype(np.int64).sum()) for a, b in bounds]
    assert max(per) - min(per) <= 2 * int(d["len"].max())


def test_shard_bounds_properties():
    assert wdist.shard_bounds(10, 3, 0) == (0, 3)
    assert wdist.shard_bounds(10, 3, 2) == (6, 10)
    rng = np.random.default_rng(0)
    for world in (1, 2, 4, 8):
        lens = np.where(rng.random(10001) < 0.5, 64, 9000)
        b = wdist.shard_bounds_by_bytes(lens, world)
        assert b[0][0] == 0 and b[-1][1] == lens.size
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        per = [int(lens[x:y].sum()) for x, y in b]
        assert max(per) - min(per) <= 2 * 9000
    # degenerate: more ranks than packets
    b = wdist.shard_bounds_by_bytes([100, 100], 4)
    assert sum(y - x for x, y in b) == 2


def test_hash_is_split_invariant():
    v = torch.randint(0, 65536, (1000,), dtype=torch.int32).to(torch.uint16)
    whole = wdist.result_hash(v, 0)
    parts = (wdist.result_hash(v[:300], 0) + wdist.result_hash(v[300:], 300)) % wdist.HASH_MOD
    assert whole == parts == exact_hash(v.to(torch.int32).numpy(), 0)


def test_hash_exact_at_large_shards_and_offsets():
    """Shard sizes and offsets where a plain int64 sum of (index * value)
    would wrap (2^22 packets per rank at 8 ranks): block sums and
    20-bit index halves keep it exact."""
    rng = np.random.default_rng(3)
    v = torch.from_numpy(rng.integers(60000, 65536, 1 << 22).astype(np.int32)).to(torch.uint16)
    for off in (0, 7 << 22, (1 << 39) + 1):
        vv = v.to(torch.int64) + 1
        i = torch.arange(vv.numel(), dtype=torch.int64)
        # exact reference: sum (off+1+i) v_i = (off+1) sum v_i + sum i v_i, each
        # int64 sum < 2^61 here, combined as Python integers
        ref = ((off + 1) * int(vv.sum()) + int((vv * i).sum())) % wdist.HASH_MOD
        assert wdist.result_hash(v, off) == ref
    # split invariance across a 2^24 block boundary
    w = v[: (1 << 22)]
    assert (wdist.result_hash(w[:12345], 5 << 30) + wdist.result_hash(w[12345:], (5 << 30) + 12345)) % \
        wdist.HASH_MOD == wdist.result_hash(w, 5 << 30)


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py --gpus 2 with RCCL and fewer visible GPUs exits non-zero
    before touching a device (the parent never initialises the GPU)."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "WG_DIST_BACKEND")}
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "GPU(s) visible" in r.stderr


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_config4_strong_shards(world):
    """bench.py's config 4 strong companion: ONE 4 M-packet bimodal batch
    split by bytes; every rank's shard buffer starts at the 16-B-aligned
    global byte its synth_fill counter base needs, its descriptors rebased
    onto it, so the shards together are the N = 1 batch; per-rank byte
    totals within one 9000-B packet of each other."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    lens, offs = bench.config4_lengths()
    assert lens.size == 1 << 22 and set(np.unique(lens)) == {64, 9000}
    bounds = wdist.shard_bounds_by_bytes(lens, world)
    assert bounds[0][0] == 0 and bounds[-1][1] == lens.size
    per = [int(lens[a:b].sum()) for a, b in bounds]
    assert sum(per) == int(lens.sum()) and max(per) - min(per) <= 9000
    for a, b in bounds:
        base = int(offs[a]) & ~15
        assert base % 16 == 0 and 0 <= int(offs[a]) - base < 16
        rel = offs[a:b] - base
        assert rel[0] < 16 and np.all(np.diff(rel) == lens[a:b - 1])
