"""bench.py's CPU-baseline leg: the oracle's worker pinning (oracle/orc_pin.h)
and its persistent worker pool (oracle/csum_oracle.c run_parallel).

Regression for round 4's collapsed baselines: workers used to be pinned by
their handle after creation, and a worker that had already finished carries
TID 0 in its handle, so sched_setaffinity(0) pinned the *calling* thread —
the next quiet_cpus() pick then saw a one-CPU mask and every later
repetition ran 16 workers on one core.  Test infrastructure only."""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import oracle  # noqa: E402


def _small_batch(n=4096):
    buf = np.random.default_rng(7).integers(0, 256, n * 64, dtype=np.uint8)
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = np.arange(n) * 64
    d["len"] = 64
    return buf, d


def test_parallel_calls_leave_the_caller_unpinned():
    buf, d = _small_batch()
    before = os.sched_getaffinity(0)
    ref = oracle.verify_desc(buf, d, 1)
    for _ in range(300):  # millisecond jobs: workers finish before the caller moves on
        got = oracle.verify_desc(buf, d, 4)
        assert os.sched_getaffinity(0) == before
    assert all(np.array_equal(a, b) for a, b in zip(ref, got))


def test_pool_follows_the_picked_cpus():
    buf, d = _small_batch()
    ref = oracle.verify_desc(buf, d, 1)
    saved = os.environ.get("ORC_CPUS")
    try:
        cpus = sorted(os.sched_getaffinity(0))
        for pick in (cpus[:2], cpus[-2:], cpus[:1]):  # a new list rebuilds the pool
            os.environ["ORC_CPUS"] = ",".join(map(str, pick))
            got = oracle.verify_desc(buf, d, 3)
            assert all(np.array_equal(a, b) for a, b in zip(ref, got))
        q = oracle.quiet_cpus(min(4, len(cpus)))
        assert len(q["cpus"]) == min(4, len(cpus)) and len(set(q["cpus"])) == len(q["cpus"])
    finally:
        if saved is None:
            os.environ.pop("ORC_CPUS", None)
        else:
            os.environ["ORC_CPUS"] = saved


def test_quiet_cpus_deals_l3_domains_round_robin():
    """the all-core leg's CPUs are dealt over the L3
    domains (CCDs) before a domain gets a second worker, one per physical
    core; the result names the domains it used."""
    cpus = sorted(os.sched_getaffinity(0))
    doms = {}
    for c in cpus:
        doms.setdefault(oracle._l3_of(c), set()).add(oracle._core_of(c))
    n = min(len(cpus), 16)
    q = oracle.quiet_cpus(n)
    assert len(q["cpus"]) == n and len(set(q["cpus"])) == n
    used = q["l3_domains"]
    assert sum(len(v) for v in used.values()) == n
    # no domain holds two workers while another holds none (when cores allow)
    if n <= len(doms):
        assert len(used) == n
    counts = [len(v) for v in used.values()]
    assert max(counts) - min(counts) <= 1 or n > sum(len(v) for v in doms.values())


def test_read_probe_and_pool_stats():
    """The read probe sums the buffer's whole 4-KiB blocks (the same word sum
    with 1 or 3 workers), and the pool reports one busy time per worker."""
    buf = np.random.default_rng(9).integers(0, 256, (1 << 20) + 100, dtype=np.uint8)
    blocks = buf[: buf.size // 4096 * 4096].view(np.uint64)
    want = int(blocks.sum(dtype=np.uint64))
    assert oracle.read_probe(buf, 1) == want
    saved = os.environ.get("ORC_CPUS")
    try:
        cpus = sorted(os.sched_getaffinity(0))
        os.environ["ORC_CPUS"] = ",".join(map(str, cpus[:3]))
        oracle.pool_stats_reset()
        assert oracle.read_probe(buf, 3) == want
        st = oracle.pool_stats()
        assert len(st) == min(3, len(cpus)) and all(calls == 1 and busy > 0 for busy, calls in st)
    finally:
        if saved is None:
            os.environ.pop("ORC_CPUS", None)
        else:
            os.environ["ORC_CPUS"] = saved
