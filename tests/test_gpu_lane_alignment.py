"""Small packets whose start alignment is the same across a wave.

The lane paths (one packet per lane: the split descriptor kernel's small
role, the walking and compacting verify kernels) load a packet's 16-B-aligned
window and realign it by the packet's dword offset q4 = (address & 15) >> 2
and byte offset address & 3 (`lane_realign`, csrc/l4csum.hip).  When q4 is
the same in every lane the wave takes one scalar branch (a straight-line copy
per q4), otherwise bit-mask selects: random offsets (test_gpu_l4.py,
test_verify_gates.py) reach the select form almost always, so this file puts
whole batches, and whole 64-descriptor runs, at each of the 16 alignments.
The split kernel's small packets are checked both loaded by the wave
together (lane_coop 1, coop_chunks) and by their own lanes (0).
Config 4's 64-B packets (8-B aligned between 9,000-B ones) are q4 0 and 2.

Checked against the oracle: calc_l4_checksum (checksum.cpp:8-36) and
checksum (include/netio/checksum.hpp:146-149) per descriptor, and the verify
gates (include/worker/evaluator.hpp:112-149), under every kernel choice."""
import numpy as np
import pytest

import oracle
import pktbuild

pytestmark = pytest.mark.gpu

STRIDE = 80  # a multiple of 16, > 64: every packet of a run at one alignment


def _wga():
    import wireglider_amd

    return wireglider_amd


def _small_packets(rng, n):
    pkts, fam = [], []
    for _ in range(n):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        hl = (40 if v6 else 20) + (20 if tcp else 8)
        al = 16 if v6 else 4
        plen = int(rng.integers(0, 65 - hl))
        p = bytearray(pktbuild.build(v6, tcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        k = int(rng.integers(0, 8))
        if k == 0:
            p[int(rng.integers(0, len(p)))] ^= 1 << int(rng.integers(0, 8))
        elif k == 1:
            p = p[: int(rng.integers(0, len(p) + 1))]
        pkts.append(bytes(p))
        fam.append((v6, tcp))
    return pkts, fam


def _layout(rng, pkts, fam, align_of_run):
    """Packet k at run (k // 64)'s alignment; the gaps hold random bytes."""
    n = len(pkts)
    offs = np.array([k * STRIDE + align_of_run(k // 64) for k in range(n)], dtype=np.uint64)
    buf = rng.integers(0, 256, n * STRIDE + 32, dtype=np.uint8)
    for o, p in zip(offs, pkts):
        buf[int(o):int(o) + len(p)] = np.frombuffer(p, np.uint8)
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = offs
    d["len"] = [len(p) for p in pkts]
    d["flags"] = [(1 if v6 else 0) | (2 if tcp else 0) for v6, tcp in fam]
    d["csum_start"] = [40 if v6 else 20 for v6, _ in fam]
    return buf, d


def _cases(seed):
    rng = np.random.default_rng(seed)
    out = []
    for a in range(16):  # the whole batch at one alignment
        pkts, fam = _small_packets(rng, 64 * 12 + 5)
        out.append((f"batch@{a}", *_layout(rng, pkts, fam, lambda r, a=a: a)))
    pkts, fam = _small_packets(rng, 64 * 48 + 17)  # each 64-descriptor run at its own alignment
    out.append(("runs", *_layout(rng, pkts, fam, lambda r: (r * 5 + 3) & 15)))
    return out


def _to_dev(buf, d, dev):
    import torch

    tb = torch.from_numpy(buf).to(dev)  # 256-B aligned allocation: offset & 15 is the address's
    td = torch.from_numpy(np.ascontiguousarray(d).view(np.int64).reshape(-1, 2).copy()).to(dev)
    assert tb.data_ptr() % 16 == 0
    return tb, td


@pytest.mark.parametrize("l4_small,lane_coop", [(0, 1), (5, 1), (5, 0)])
def test_l4_desc_uniform_alignment(gpu, l4_small, lane_coop):
    import torch

    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("l4_small", "l4_coop", "lane_coop")}
    try:
        wga.tune_set("l4_small", l4_small)
        wga.tune_set("l4_coop", 0)
        wga.tune_set("lane_coop", lane_coop)
        for name, buf, d in _cases(71):
            tb, td = _to_dev(buf, d, gpu)
            out = wga.calc_l4_checksum_desc(tb, td)
            plain = wga.checksum_desc(tb, td)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy(), oracle.l4_desc(buf, d), err_msg=name)
            np.testing.assert_array_equal(plain.cpu().numpy(), oracle.checksum_desc(buf, d), err_msg=name)
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)


@pytest.mark.parametrize("verify_small", [0, 6, 7, 8])
def test_verify_desc_uniform_alignment(gpu, verify_small):
    """Three calls per batch on one fresh stream: with verify_small = 7 the
    first runs the walking kernel (consecutive layout) and the later ones the
    kernel the sample picks; 6 the compacting path, 8 the walking kernel
    (spread layout), 0 the wave kernel."""
    import torch

    wga = _wga()
    saved = wga.tune_get("verify_small")
    try:
        wga.tune_set("verify_small", verify_small)
        for name, buf, d in _cases(72):
            tb, td = _to_dev(buf, d, gpu)
            want_v, want_l4 = oracle.verify_desc(buf, d)
            s = torch.cuda.Stream(gpu)
            with torch.cuda.stream(s):
                for call in range(3):
                    v, l4 = wga.verify_desc(tb, td)
                    s.synchronize()
                    np.testing.assert_array_equal(v.cpu().numpy(), want_v, err_msg=f"{name} call {call}")
                    np.testing.assert_array_equal(l4.cpu().numpy(), want_l4, err_msg=f"{name} call {call}")
    finally:
        wga.tune_set("verify_small", saved)
