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
    totals.  Every range boundary is the first packet whose byte prefix sum
    reaches rank * total / world, so the largest imbalance is one packet."""
    import numpy as np

    lens = np.asarray(lengths, dtype=np.int64)
    n = lens.size
    if world < 1:
        raise ValueError("world must be >= 1")
    csum = np.concatenate([[0], np.cumsum(lens)])
    total = int(csum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        cuts.append(int(np.searchsorted(csum, target, side="left")))
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):  # monotone
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def result_hash(results, global_offset: int):
    """Order-independent hash of a shard of uint16 results: sum over packets
    of (global_index + 1) * (value + 1) mod 2^61-1, as an int64 tensor; the
    all-reduced (SUM then mod) hash equals the hash of the whole array."""
    import torch

    v = results.to(torch.int64) + 1
    idx = torch.arange(global_offset + 1, global_offset + 1 + v.numel(), dtype=torch.int64, device=v.device)
    # products < 2^16 * 2^40 for batches below 2^40 packets: no overflow
    return ((v * idx) % HASH_MOD).sum() % HASH_MOD


def allreduce_hash(local_hash, group=None):
    import torch
    import torch.distributed as dist

    t = local_hash.clone().reshape(1)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item()) % HASH_MOD


def gather_results(local, counts: Sequence[int], group=None):
    """All-gather variable-size uint16 shards into the full result array
    (padded all_gather, then trimmed).  `counts[r]` = packets of rank r."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local.clone()
    mx = max(counts)
    buf = torch.zeros(mx, dtype=torch.int32, device=local.device)
    buf[: local.numel()] = local.to(torch.int32)
    parts = [torch.empty_like(buf) for _ in counts]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(torch.uint16)


def max_over_ranks(x: float, device=None, group=None) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
