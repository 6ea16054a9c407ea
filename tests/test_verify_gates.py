"""Decap verify gates: oracle restatement pinned by the
reference's own decap tests, and GPU parity of wg_verify_desc.

Reference semantics: include/worker/evaluator.hpp:112-149 (evaluate_packet),
worker/evaluator.cpp:14-58 (fill_fk_ip4 / fill_fk_ip6), evaluator.hpp:59-65
and 89-94 (TCP / UDP checksum gates).  Reference tests restated:
tests/test-flowkey-own.cpp:170-200 "coalesceItemInvalidCSum" (a flipped L4
checksum -> GRO_NOADD) and :456-501 "DecapBatch invalid packets".
"""
import struct

import numpy as np
import pytest

import oracle
import pktbuild

V = oracle
OK = V.V_IP_OK | V.V_L4_OK


def tcp4(n=100, seq=1):
    return bytearray(pktbuild.make_tcp(False, "192.0.2.1", 1, "192.0.2.2", 1, 0x10, n, seq))


def udp4(n=100):
    return bytearray(pktbuild.make_udp(False, "192.0.2.1", 1, "192.0.2.2", 1, n))


def tcp6(n=100):
    return bytearray(pktbuild.make_tcp(True, "2001:db8::1", 1, "2001:db8::2", 1, 0x10, n, 1))


def udp6(n=100):
    return bytearray(pktbuild.make_udp(True, "2001:db8::1", 1, "2001:db8::2", 1, n))


def flip_l4(p, isv6, istcp):
    off = (40 if isv6 else 20) + (16 if istcp else 6)
    p[off] ^= 0xFF
    p[off + 1] ^= 0xFF
    return p


def test_valid_packets_pass():
    assert V.verify(tcp4())[0] == OK | V.V_TCP
    assert V.verify(udp4())[0] == OK | V.V_UDP
    assert V.verify(tcp6())[0] == OK | V.V_TCP | V.V_V6
    assert V.verify(udp6())[0] == OK | V.V_UDP | V.V_V6


def test_coalesce_item_invalid_csum():
    # tests/test-flowkey-own.cpp:170-200: flipped L4 checksum -> not coalesced
    for mk, v6, tcp in ((tcp4, False, True), (udp4, False, False), (tcp6, True, True), (udp6, True, False)):
        v, c = V.verify(flip_l4(mk(), v6, tcp))
        assert v & V.V_IP_OK and not v & V.V_L4_OK and c != 0


def test_invalid_packets():
    # tests/test-flowkey-own.cpp:456-501
    assert not V.verify(tcp4()[:40])[0] & V.V_IP_OK         # tcp4 too short (ip_len mismatch)
    assert not V.verify(udp4()[:28])[0] & V.V_IP_OK         # udp4 too short
    assert not V.verify(tcp6()[:60])[0] & V.V_IP_OK         # tcp6 too short (plen mismatch)
    assert not V.verify(udp6()[:48])[0] & V.V_IP_OK         # udp6 too short
    assert V.verify(bytes(1))[0] == 0                        # invalid IP version / size
    p = tcp4()
    p[0] |= 0xF                                              # invalid IP header len
    assert not V.verify(p)[0] & V.V_IP_OK
    p = tcp4()
    p[9] = 47                                                # ip4 invalid protocol (GRE)
    p[10:12] = b"\0\0"
    c = oracle.checksum(np.frombuffer(bytes(p[:20]), np.uint8), 0)
    p[10:12] = struct.pack("<H", c)
    assert V.verify(p)[0] == V.V_IP_OK
    p = tcp6()
    p[6] = 47                                                # ip6 invalid protocol
    assert V.verify(p)[0] == V.V_IP_OK | V.V_V6


def test_ip_header_gates():
    p = tcp4()
    p[6] |= 0x20  # MF set -> fragment (evaluator.cpp:24)
    assert not V.verify(p)[0] & V.V_IP_OK
    p = tcp4()
    p[6] = 0x40  # DF alone is fine, but it changes the header checksum
    assert not V.verify(p)[0] & V.V_IP_OK
    p = tcp4()
    p[8] ^= 1  # TTL change -> header checksum fails (evaluator.cpp:27)
    assert not V.verify(p)[0] & V.V_IP_OK
    # L4 length floors: TCP needs > 20 bytes after the IP header, UDP > 8
    p = tcp4(0)
    v, c = V.verify(p)
    assert v == V.V_IP_OK | V.V_TCP and c == 0
    p = udp4(0)
    assert V.verify(p)[0] == V.V_IP_OK | V.V_UDP


def random_verify_batch(rng, n):
    pkts = []
    for _ in range(n):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        plen = int(rng.choice([0, 1, 7, 8, 9, 20, 21, int(rng.integers(0, 3000))]))
        al = 16 if v6 else 4
        p = bytearray(pktbuild.build(v6, tcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        k = int(rng.integers(0, 10))
        if k == 0:
            flip_l4(p, v6, tcp) if len(p) >= (40 if v6 else 20) + (18 if tcp else 8) else None
        elif k == 1:
            p[int(rng.integers(0, len(p)))] ^= 1 << int(rng.integers(0, 8))
        elif k == 2:
            p = p[: int(rng.integers(0, len(p) + 1))]
        elif k == 3 and not v6:
            p[6] |= 0x20
        elif k == 4:
            p[6 if v6 else 9] = int(rng.choice([1, 47, 58, 132]))
        pkts.append(bytes(p))
    return pkts


def pack(pkts, rng):
    offs, o = [], int(rng.integers(0, 16))
    for p in pkts:
        offs.append(o)
        o += len(p) + int(rng.integers(0, 5))
    buf = np.zeros(o + 16, np.uint8)
    for off, p in zip(offs, pkts):
        buf[off:off + len(p)] = np.frombuffer(p, np.uint8)
    d = np.zeros(len(pkts), dtype=oracle.PKT_DESC)
    d["offset"], d["len"] = offs, [len(p) for p in pkts]
    return buf, d


def test_oracle_verify_desc_matches_scalar():
    rng = np.random.default_rng(3)
    pkts = random_verify_batch(rng, 500)
    buf, d = pack(pkts, rng)
    verdict, l4 = oracle.verify_desc(buf, d, threads=3)
    for i, p in enumerate(pkts):
        assert (verdict[i], l4[i]) == V.verify(p)


VERIFY_VARIANTS = [{"verify_small": 0}, {"verify_small": 6}, {"verify_small": 6, "verify_k2min": 8},
                   {"verify_small": 7}, {"verify_small": 7, "verify_auto_t": 64}, {"verify_small": 8}]


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", VERIFY_VARIANTS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_gpu_verify_parity(gpu, knobs):
    import torch

    import wireglider_amd as wga

    saved = {k: wga.tune_get(k) for k in knobs}
    for k, v in knobs.items():
        wga.tune_set(k, v)

    rng = np.random.default_rng(11)
    pkts = random_verify_batch(rng, 20000)
    buf, d = pack(pkts, rng)
    dbuf = torch.from_numpy(buf).to(gpu)
    dd = torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu)
    verdict, l4 = wga.verify_desc(dbuf, dd)
    torch.cuda.synchronize()
    for k, v in saved.items():
        wga.tune_set(k, v)
    ev, el4 = oracle.verify_desc(buf, d)
    np.testing.assert_array_equal(verdict.cpu().numpy(), ev)
    np.testing.assert_array_equal(l4.cpu().numpy(), el4)
    assert (ev & OK == OK).mean() > 0.3 and (ev & OK != OK).mean() > 0.2  # both outcomes exercised


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", VERIFY_VARIANTS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_gpu_verify_size_gate(gpu, knobs):
    """Packets at and past the 65535-byte size gate (evaluator.hpp:118-121):
    the gate fails, but the V6 verdict bit still follows the version nibble;
    mixed with maximum-size valid packets and short ones."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(12)
    pkts = []
    for v6 in (False, True):
        for tcp in (False, True):
            hl = (40 if v6 else 20) + (20 if tcp else 8)
            al = 16 if v6 else 4
            addr = lambda: rng.integers(0, 256, al, dtype=np.uint8).tobytes()  # noqa: E731
            pay = lambda k: rng.integers(0, 256, k, dtype=np.uint8).tobytes()  # noqa: E731
            big = pktbuild.build(v6, tcp, pay(65535 - hl), addr(), addr())  # exactly 65535 B: passes the gate
            pkts.append(big)
            for extra in (1, 4465, 70000 - 65535):  # past the gate
                pkts.append(big + pay(extra))
            small = pktbuild.build(v6, tcp, pay(1400), addr(), addr())
            pkts += [small, small[:31], small[:33]]
    buf, d = pack(pkts, rng)
    saved = {k: wga.tune_get(k) for k in knobs}
    for k, v in knobs.items():
        wga.tune_set(k, v)
    try:
        verdict, l4 = wga.verify_desc(torch.from_numpy(buf).to(gpu),
                                      torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu))
        torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)
    ev, el4 = oracle.verify_desc(buf, d)
    np.testing.assert_array_equal(verdict.cpu().numpy(), ev)
    np.testing.assert_array_equal(l4.cpu().numpy(), el4)
    assert np.count_nonzero(ev & V.V_V6) == sum(1 for p in pkts if p[0] >> 4 == 6)  # oversized v6 still report V6
    assert (ev[0::7] & OK == OK).all()  # the 65535-byte packets pass


@pytest.mark.gpu
def test_gpu_verify_high_addresses(gpu):
    """Packets placed on both sides of bit 31 and of 4 GiB in a 4.3 GB batch
    buffer (64-bit descriptor offsets, lane-level address arithmetic)."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(31)
    pkts = random_verify_batch(rng, 48)
    span = (1 << 32) + (1 << 22)
    big = torch.zeros(span, dtype=torch.uint8, device=gpu)
    # 10 slots of 3,100 B per base (packets < 3,100 B); the bases far enough
    # apart that no two packets overlap, two of them straddling bit 31 / 4 GiB
    bases = [0, (1 << 31) - 15500, (1 << 31) + 16000, (1 << 32) - 15500, (1 << 32) + 16000]
    d = np.zeros(len(pkts), dtype=oracle.PKT_DESC)
    host_buf, hd = pack(pkts, rng)  # compact copy for the oracle
    assert max(len(p) for p in pkts) + 16 < 3100
    for k, p in enumerate(pkts):
        o = bases[k % len(bases)] + (k // len(bases)) * 3100 + int(rng.integers(0, 16))
        d[k]["offset"], d[k]["len"] = o, len(p)
        if len(p):
            big[o:o + len(p)] = torch.from_numpy(np.frombuffer(p, np.uint8).copy()).to(gpu)
    verdict, l4 = wga.verify_desc(big, torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu))
    torch.cuda.synchronize()
    ev, el4 = oracle.verify_desc(host_buf, hd)
    np.testing.assert_array_equal(verdict.cpu().numpy(), ev)
    np.testing.assert_array_equal(l4.cpu().numpy(), el4)
    del big
    torch.cuda.empty_cache()


def interleaved_batch(rng, n):
    """Small (<= 64 B) and long packets interleaved in runs of 1-9, so
    4-descriptor groups are all-small, all-long and mixed at every position;
    valid and corrupted packets of every family, 0-B and 1-B packets, and
    packets of exactly 64 and 65 bytes (the lane / wave boundary)."""
    pkts = []
    small = True
    while len(pkts) < n:
        for _ in range(int(rng.integers(1, 10))):
            v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
            hl = (40 if v6 else 20) + (20 if tcp else 8)
            al = 16 if v6 else 4
            if small:
                plen = int(rng.integers(0, max(1, 65 - hl)))
            else:
                plen = int(rng.choice([65 - hl, 66 - hl, int(rng.integers(65 - hl, 2000))]))
            p = bytearray(pktbuild.build(v6, tcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                         rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                         rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
            k = int(rng.integers(0, 8))
            if k == 0:
                p[int(rng.integers(0, len(p)))] ^= 1 << int(rng.integers(0, 8))
            elif k == 1 and small:
                p = p[: int(rng.integers(0, 3))]
            pkts.append(bytes(p))
        small = not small
    return pkts[:n]


@pytest.mark.gpu
@pytest.mark.parametrize("knobs", VERIFY_VARIANTS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
def test_gpu_verify_interleaved(gpu, knobs):
    """Mixed batches whose small and long packets interleave (the two-role
    kernels split every group by packet size)."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(13)
    pkts = interleaved_batch(rng, 12001)
    assert any(len(p) == 64 for p in pkts) and any(len(p) == 65 for p in pkts)
    buf, d = pack(pkts, rng)
    saved = {k: wga.tune_get(k) for k in knobs}
    for k, v in knobs.items():
        wga.tune_set(k, v)
    try:
        verdict, l4 = wga.verify_desc(torch.from_numpy(buf).to(gpu),
                                      torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu))
        torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)
    ev, el4 = oracle.verify_desc(buf, d)
    np.testing.assert_array_equal(verdict.cpu().numpy(), ev)
    np.testing.assert_array_equal(l4.cpu().numpy(), el4)
    assert (ev & OK == OK).mean() > 0.3


@pytest.mark.gpu
@pytest.mark.parametrize("seg", [1, 7, 20, 28, 40, 48, 60, 63, 64, 65, 100, 1500, 1504, 9000])
def test_gpu_verify_uniform(gpu, seg):
    """wg_verify_uniform (a PacketBatch, no descriptors) equals the oracle on
    the same segments: valid and corrupted packets of every family whose
    length is the segment size, a short last segment, every alignment of
    the batch start, both kernels (segment size <= 64: a lane per packet)."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(seg)
    n = 3001
    pkts = []
    for _ in range(n):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        hl = (40 if v6 else 20) + (20 if tcp else 8)
        al = 16 if v6 else 4
        if seg >= hl:
            p = bytearray(pktbuild.build(v6, tcp, rng.integers(0, 256, seg - hl, dtype=np.uint8).tobytes(),
                                         rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                         rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
            if rng.integers(0, 5) == 0:
                p[int(rng.integers(0, seg))] ^= 1 << int(rng.integers(0, 8))
        else:
            p = bytearray(rng.integers(0, 256, seg, dtype=np.uint8).tobytes())
        pkts.append(bytes(p))
    for lead in (0, 1, 3, 8):
        total = n * seg - int(rng.integers(0, seg))  # a short last segment
        buf = np.zeros(lead + n * seg + 16, np.uint8)
        buf[lead:lead + n * seg] = np.frombuffer(b"".join(pkts), np.uint8)
        dbuf = torch.from_numpy(buf).to(gpu)
        verdict, l4 = wga.verify_uniform(dbuf[lead:lead + total], seg)
        torch.cuda.synchronize()
        m = (total + seg - 1) // seg
        d = np.zeros(m, dtype=oracle.PKT_DESC)
        d["offset"] = lead + np.arange(m, dtype=np.uint64) * seg
        d["len"] = np.minimum(seg, total - np.arange(m) * seg)
        ev, el4 = oracle.verify_desc(buf, d)
        np.testing.assert_array_equal(verdict.cpu().numpy(), ev, err_msg=f"lead {lead}")
        np.testing.assert_array_equal(l4.cpu().numpy(), el4, err_msg=f"lead {lead}")
        if seg >= 60:
            assert (ev & OK == OK).mean() > 0.5


def _verify_calls(wga, torch, gpu, batches, knobs, stream=None):
    """wg_verify_desc over each (buf, desc) in order on one stream under knobs;
    returns the host copies of every call's verdicts and L4 results."""
    saved = {k: wga.tune_get(k) for k in knobs}
    for k, v in knobs.items():
        wga.tune_set(k, v)
    out = []
    try:
        ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            for buf, d in batches:
                verdict, l4 = wga.verify_desc(torch.from_numpy(buf).to(gpu),
                                              torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu))
                out.append((verdict, l4))
        torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)
    return [(v.cpu().numpy(), x.cpu().numpy()) for v, x in out]


@pytest.mark.gpu
def test_gpu_verify_auto_switches(gpu):
    """The default wg_verify_desc (verify_small = 7) picks its kernel per call
    from the size mix the previous call on the stream sampled (the walking
    kernel on a stream's first call and after an all-small sample): all-small,
    all-long and interleaved batches back to back, each followed by a
    different one (every call then runs on a stale sample, including the
    compacting path's long kernel sized for no long packets at all, with a
    1-block-per-shard minimum grid), on the default stream and on a fresh side
    stream — every call's results equal the oracle's."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(14)

    def sized(n, lo, hi):
        pkts = []
        for _ in range(n):
            v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
            hl = (40 if v6 else 20) + (20 if tcp else 8)
            al = 16 if v6 else 4
            plen = int(rng.integers(max(0, lo - hl), max(1, hi - hl)))
            pkts.append(pktbuild.build(v6, tcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                       rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                       rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        return pkts

    kinds = {"small": sized(9000, 40, 65), "long": sized(9000, 65, 1600), "mixed": interleaved_batch(rng, 9001)}
    packed = {k: pack(v, rng) for k, v in kinds.items()}
    order = ["small", "long", "small", "mixed", "mixed", "long", "long", "small", "small", "mixed", "long"]
    expect = {k: oracle.verify_desc(*packed[k]) for k in kinds}
    for stream in (None, torch.cuda.Stream(gpu)):
        got = _verify_calls(wga, torch, gpu, [packed[k] for k in order],
                            {"verify_small": 7, "verify_auto_t": 4, "verify_k2min": 8}, stream)
        for k, (v, x) in zip(order, got):
            np.testing.assert_array_equal(v, expect[k][0], err_msg=k)
            np.testing.assert_array_equal(x, expect[k][1], err_msg=k)
    assert (expect["long"][0] & OK == OK).mean() > 0.9 and (expect["small"][0] & OK == OK).mean() > 0.9


@pytest.mark.gpu
def test_gpu_verify_walk_consecutive_layout(gpu):
    """All-small batches back to back on one stream: from the third call the
    default picks the walking kernel in its consecutive layout (each wave's 64
    descriptors in a row); a batch whose size is no multiple of 64, packets of
    0-64 bytes at odd offsets, and the same batch's descriptors reversed (the
    lanes' packets then run backwards through memory) equal the oracle."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(16)
    pkts = []
    for _ in range(70001):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        hl = (40 if v6 else 20) + (20 if tcp else 8)
        if hl <= 64 and rng.integers(0, 8):
            al = 16 if v6 else 4
            pkts.append(pktbuild.build(v6, tcp, rng.integers(0, 256, int(rng.integers(0, 65 - hl)), dtype=np.uint8)
                                       .tobytes(), rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                       rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        else:
            pkts.append(rng.integers(0, 256, int(rng.integers(0, 65)), dtype=np.uint8).tobytes())
    buf, d = pack(pkts, rng)
    rev = (buf, d[::-1].copy())
    batches = [(buf, d), (buf, d), (buf, d), rev, rev]
    got = _verify_calls(wga, torch, gpu, batches, {"verify_small": 7})
    for (b, dd), (v, x) in zip(batches, got):
        ev, el4 = oracle.verify_desc(b, dd)
        np.testing.assert_array_equal(v, ev)
        np.testing.assert_array_equal(x, el4)
    ev, _ = oracle.verify_desc(buf, d)
    assert (ev & OK == OK).mean() > 0.5


@pytest.mark.gpu
def test_gpu_verify_compact_grows(gpu):
    """The compacting path's entry lists grow with the batch (a batch larger
    than every earlier one on the stream), and a 1-packet batch after it."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(15)
    batches = [pack(interleaved_batch(rng, n), rng) for n in (300, 70001, 1)]
    got = _verify_calls(wga, torch, gpu, batches, {"verify_small": 6})
    for (buf, d), (v, x) in zip(batches, got):
        ev, el4 = oracle.verify_desc(buf, d)
        np.testing.assert_array_equal(v, ev)
        np.testing.assert_array_equal(x, el4)


@pytest.mark.gpu
@pytest.mark.parametrize("warm", [False, True])
def test_gpu_verify_under_graph_capture(gpu, warm):
    """wg_verify_desc captured into a HIP graph (torch.cuda.graph) on a side
    stream — with no per-stream state yet (warm False) or after eager calls
    gave the stream a sample (warm True): captured calls take a stateless
    kernel (no entry lists, no counter sets frozen into the graph, nothing
    allocated while capturing), and every replay equals the oracle (ADVICE
    r03: a replayed compacting path reused one counter set without zeroing
    it; a missing state fell through to a kernel the comment did not name)."""
    import torch

    import wireglider_amd as wga

    rng = np.random.default_rng(16 + warm)
    for pkts in (interleaved_batch(rng, 5000), random_verify_batch(rng, 3000),
                 [p for p in interleaved_batch(rng, 6000) if len(p) <= 64][:3000]):
        buf, d = pack(pkts, rng)
        dbuf = torch.from_numpy(buf).to(gpu)
        dd = torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(gpu)
        n = len(d)
        verdict = torch.empty(n, dtype=torch.uint8, device=gpu)
        l4 = torch.empty(n, dtype=torch.uint16, device=gpu)
        s = torch.cuda.Stream(gpu)
        if warm:
            with torch.cuda.stream(s):
                for _ in range(3):  # the stream's state and sample exist before the capture
                    wga.verify_desc(dbuf, dd, verdict=verdict, l4=l4)
            torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            wga.verify_desc(dbuf, dd, verdict=verdict, l4=l4)
        ev, el4 = oracle.verify_desc(buf, d)
        for _ in range(3):
            verdict.zero_()
            l4.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(verdict.cpu().numpy(), ev)
            np.testing.assert_array_equal(l4.cpu().numpy(), el4)
