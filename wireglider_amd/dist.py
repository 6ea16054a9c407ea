"""Multi-GPU sharding of packet batches.

Every packet (and every GSO super-buffer) is independent — calc_l4_checksum
is pure (reference checksum.cpp:8-36) — so a batch shards into contiguous
packet ranges, one per rank (one process per GPU), with NO collective on the
data path.  Collectives are used only around it:
  - gather_results(): all-gather of the 2-byte results (RCCL over xGMI on
    the "nccl" backend; gloo in CPU tests);
  - result_hash(): an order-independent hash of the results, all-reduced,
    for the bit-exact check against a reference hash;
  - max_over_ranks(): the max of a timing value (bench.py).
Shards are balanced by BYTES, not packet counts (config 4-style mixes).
Every helper runs its collective whenever a process group exists, even of
one rank (bench.py --force-dist: the RCCL code path exercised on a one-GPU
box); without a group they return the local answer.
"""
from __future__ import annotations

from typing import Sequence

HASH_MOD = (1 << 61) - 1  # Mersenne prime: exact in int64 arithmetic below


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, count-balanced packet range of `rank` (uniform batches)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return n * rank // world, n * (rank + 1) // world


def shard_bounds_by_bytes(lengths: Sequence[int], world: int) -> list[tuple[int, int]]:
    """Split packets 0..n-1 into `world` contiguous ranges of near-equal byte
    totals.  Each boundary is one of the two packet boundaries around
    rank * total / world (the prefix sums just below and at-or-above it);
    of those 2^(world-1) choices (world <= 12; else the nearer one each) the
    one with the smallest spread of shard byte totals wins, so a shard is off
    the mean by at most about one packet."""
    import itertools

    import numpy as np

    lens = np.asarray(lengths, dtype=np.int64)
    n = lens.size
    if world < 1:
        raise ValueError("world must be >= 1")
    csum = np.concatenate([[0], np.cumsum(lens)])
    total = int(csum[-1])
    cands = []
    for r in range(1, world):
        target = total * r // world
        j = int(np.searchsorted(csum, target, side="left"))
        lo_c, hi_c = max(j - 1, 0), min(j, n)
        if world > 12:  # the nearer boundary only
            near = lo_c if target - int(csum[lo_c]) <= int(csum[hi_c]) - target else hi_c
            cands.append((near,))
        else:
            cands.append(tuple(sorted({lo_c, hi_c})))
    best, best_spread = None, None
    for choice in itertools.product(*cands) if cands else [()]:
        cuts = [0, *choice, n]
        if any(cuts[i] > cuts[i + 1] for i in range(world)):
            continue
        per = [int(csum[cuts[i + 1]] - csum[cuts[i]]) for i in range(world)]
        spread = max(per) - min(per)
        if best_spread is None or spread < best_spread:
            best, best_spread = cuts, spread
    if best is None:  # (cannot happen: the all-lower choice is monotone) fall back to count balance
        best = [n * r // world for r in range(world + 1)]
    return [(best[r], best[r + 1]) for r in range(world)]


def result_hash(results, global_offset: int) -> int:
    """Order-independent hash of a shard of uint16 results: sum over packets
    of (global_index + 1) * (value + 1) mod 2^61-1.  The per-rank hashes add
    (mod 2^61-1) to the hash of the whole array.

    Exact for any shard size and offset below 2^40: the index is split into
    20-bit halves, so each int64 product is < 2^17 * 2^20, and the shard is
    summed in blocks of 2^24 packets (block sums < 2^61); the blocks are
    combined as Python integers."""
    import torch

    v = results.reshape(-1).to(torch.int64) + 1
    total = 0
    blk = 1 << 24
    for s0 in range(0, v.numel(), blk):
        vb = v[s0 : s0 + blk]
        idx = torch.arange(global_offset + 1 + s0, global_offset + 1 + s0 + vb.numel(), dtype=torch.int64,
                           device=v.device)
        lo = int((vb * (idx & 0xFFFFF)).sum().item())
        hi = int((vb * (idx >> 20)).sum().item())
        total = (total + lo + (hi << 20)) % HASH_MOD
    return total


def allreduce_hash(local_hash: int, group=None, device=None) -> int:
    """Sum of the ranks' hashes mod 2^61-1.  Each hash is < 2^61, so eight of
    them would overflow an int64 all-reduce: the 31-bit halves are reduced
    separately (sums < 2^34) and recombined here."""
    import torch
    import torch.distributed as dist

    h = int(local_hash)
    if not dist.is_initialized():
        return h % HASH_MOD
    t = torch.tensor([h & 0x7FFFFFFF, h >> 31], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return (int(t[0].item()) + (int(t[1].item()) << 31)) % HASH_MOD


def gather_results(local, counts: Sequence[int], group=None):
    """All-gather variable-size uint16 shards into the full result array
    (padded all_gather, then trimmed).  `counts[r]` = packets of rank r.
    The shards travel as their raw bytes (a uint8 view of even length), so
    the gather moves 2 B per packet, plus the padding of the
    shorter shards up to the longest."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return local.clone()
    mx = max(counts)
    buf = torch.zeros(2 * mx, dtype=torch.uint8, device=local.device)
    buf[: 2 * local.numel()] = local.reshape(-1).contiguous().view(torch.uint8)
    parts = [torch.empty_like(buf) for _ in counts]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[: 2 * c] for p, c in zip(parts, counts)]).view(torch.uint16)


def max_over_ranks(x: float, device=None, group=None) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_gather_floats(values: Sequence[float], device=None, group=None) -> list[list[float]]:
    """Every rank's list of floats (same length on every rank), in rank
    order; [values] without a process group.  bench.py reports per-rank kernel
    and wall times with it (stragglers show up there, not in the max)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return [list(map(float, values))]
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [p.cpu().tolist() for p in parts]
