"""Pin the oracle's do_tun_gso_split restatement (worker/offload.cpp:46-216).

offload.cpp is unbuildable here (boost.endian, tdutil, fastcsum absent), so
the restatement is pinned by the reference's own assertions in
tests/test-offload.cpp:21-171 (segment size, segment count, TCP seq per
segment, for tcp4/tcp6/udp4/udp6 and the GSO_NONE "unrel" case, with
hdr_len 40/60/28/48 or the packet size) and by independent checks on every
produced segment: the IPv4 header checksum and the L4 checksum verify with
the RFC textbook implementation, the payload is the input payload in order,
FIN/PSH survive only on the last segment, and the ECN quirk (:55 vs :151)
behaves as SURVEY §8a A6 recorded it.
"""
import struct

import numpy as np
import pytest

import oracle
import pktbuild
import textbook

NEEDS_CSUM = 1
GSO_NONE, GSO_TCPV4, GSO_TCPV6, GSO_UDP_L4, GSO_ECN = 0, 1, 4, 5, 0x80


def split(pkt: bytes, **vnet):
    st, inb, out, vafter, res = oracle.gso_split(np.frombuffer(pkt, np.uint8), vnet, 131072)
    return st, inb, out, vafter, res


def tcp_seq(seg: bytes, cs: int) -> int:
    return struct.unpack(">I", seg[cs + 4:cs + 8])[0]


@pytest.mark.parametrize("hdrlen", [40, 0])
def test_tcp4(hdrlen):
    # tests/test-offload.cpp:21-47
    pkt = pktbuild.make_tcp(False, "192.0.2.1", 1, "192.0.2.2", 1, 0x18, 200, 9999)
    st, _, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_TCPV4, hdr_len=hdrlen or len(pkt),
                               gso_size=100, csum_start=20, csum_offset=16)
    assert st == 0 and res["segment_size"] == 140 and len(out) == 2 * 140
    assert tcp_seq(bytes(out[:140]), 20) == 9999
    assert tcp_seq(bytes(out[140:]), 20) == 9999 + 100


@pytest.mark.parametrize("hdrlen", [40, 0])
def test_tcp4_unrel(hdrlen):
    # tests/test-offload.cpp:49-70 (GSO_NONE: returned unsegmented)
    pkt = pktbuild.make_tcp(False, "192.0.2.1", 1, "192.0.2.2", 1, 0x19, 100, 9999)
    st, inb, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_NONE, hdr_len=hdrlen or len(pkt),
                                 gso_size=100, csum_start=20, csum_offset=16)
    assert st == 0 and res["passthrough"] == 1 and res["segment_size"] == 140 and res["out_len"] == 140
    assert tcp_seq(bytes(inb), 20) == 9999
    # in-place checksums verify (offload.cpp:56-78)
    assert oracle.checksum(inb[:20], 0) == 0
    assert textbook.l4_checksum_native(bytes(inb), False, True, 20) == 0


@pytest.mark.parametrize("hdrlen", [60, 0])
def test_tcp6(hdrlen):
    # tests/test-offload.cpp:72-97
    pkt = pktbuild.make_tcp(True, "2001:db8::1", 1, "2001:db8::2", 1, 0x18, 200, 9999)
    st, _, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_TCPV6, hdr_len=hdrlen or len(pkt),
                               gso_size=100, csum_start=40, csum_offset=16)
    assert st == 0 and res["segment_size"] == 160 and len(out) == 2 * 160
    assert tcp_seq(bytes(out[:160]), 40) == 9999
    assert tcp_seq(bytes(out[160:]), 40) == 10099


@pytest.mark.parametrize("hdrlen", [60, 0])
def test_tcp6_unrel(hdrlen):
    # tests/test-offload.cpp:99-119
    pkt = pktbuild.make_tcp(True, "2001:db8::1", 1, "2001:db8::2", 1, 0x19, 100, 9999)
    st, inb, _, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_NONE, hdr_len=hdrlen or len(pkt),
                               gso_size=100, csum_start=40, csum_offset=16)
    assert st == 0 and res["segment_size"] == 160 and res["out_len"] == 160
    assert textbook.l4_checksum_native(bytes(inb), True, True, 40) == 0


@pytest.mark.parametrize("isv6,cs,hdrlen,segsz", [(False, 20, 28, 128), (True, 40, 48, 148)])
@pytest.mark.parametrize("zero_hdrlen", [False, True])
def test_udp(isv6, cs, hdrlen, segsz, zero_hdrlen):
    # tests/test-offload.cpp:121-171
    a = ("2001:db8::1", "2001:db8::2") if isv6 else ("192.0.2.1", "192.0.2.2")
    pkt = pktbuild.make_udp(isv6, a[0], 1, a[1], 1, 200)
    st, _, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_UDP_L4,
                               hdr_len=len(pkt) if zero_hdrlen else hdrlen, gso_size=100, csum_start=cs,
                               csum_offset=6)
    assert st == 0 and res["segment_size"] == segsz and len(out) == 2 * segsz
    for k in range(2):
        seg = bytes(out[k * segsz:(k + 1) * segsz])
        assert struct.unpack(">H", seg[cs + 4:cs + 6])[0] == segsz - cs  # udp->len
        assert textbook.l4_checksum_native(seg, isv6, False, cs) == 0


def segments(out: bytes, segsz: int):
    return [out[i:i + segsz] for i in range(0, len(out), segsz)]


@pytest.mark.parametrize("isv6", [False, True])
@pytest.mark.parametrize("istcp", [False, True])
def test_random_properties(isv6, istcp):
    rng = np.random.default_rng(100 + 2 * isv6 + istcp)
    for _ in range(40):
        plen = int(rng.integers(0, 6000))
        gso = int(rng.integers(1, 1500))
        fin = int(rng.integers(0, 2))
        pkt = pktbuild.build(isv6, istcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                             rng.integers(0, 256, 16 if isv6 else 4, dtype=np.uint8).tobytes(),
                             rng.integers(0, 256, 16 if isv6 else 4, dtype=np.uint8).tobytes(),
                             seq=int(rng.integers(0, 2**32)), tcp_flags=0x18 | fin, ident=int(rng.integers(0, 65536)),
                             fill_l4=False)
        cs = 40 if isv6 else 20
        hl = cs + (20 if istcp else 8)
        gt = (GSO_TCPV6 if isv6 else GSO_TCPV4) if istcp else GSO_UDP_L4
        st, inb, out, vafter, res = split(pkt, flags=NEEDS_CSUM, gso_type=gt, hdr_len=int(rng.integers(0, 300)),
                                          gso_size=gso, csum_start=cs, csum_offset=16 if istcp else 6)
        assert st == 0 and vafter["hdr_len"] == hl
        nseg = (plen + gso - 1) // gso
        assert res["segment_size"] == hl + gso and len(out) == plen + nseg * hl
        segs = segments(bytes(out), hl + gso)
        assert len(segs) == nseg
        payload = b"".join(s[hl:] for s in segs)
        assert payload == pkt[hl:]
        for i, s in enumerate(segs):
            if not isv6:
                assert oracle.checksum(np.frombuffer(s[:20], np.uint8), 0) == 0
                assert struct.unpack(">H", s[2:4])[0] == len(s)
                assert struct.unpack(">H", s[4:6])[0] == (struct.unpack(">H", pkt[4:6])[0] + i) & 0xFFFF
            else:
                assert struct.unpack(">H", s[4:6])[0] == len(s) - 40
            assert textbook.l4_checksum_native(s, isv6, istcp, cs) == 0
            if istcp:
                assert tcp_seq(s, cs) == (tcp_seq(pkt, cs) + gso * i) & 0xFFFFFFFF
                last = i == nseg - 1
                assert (s[cs + 13] & 0x09) == ((0x08 | fin) if last else 0)
        # input prefix zeroed in place (offload.cpp:145-149)
        if not isv6:
            assert inb[10] == 0 and inb[11] == 0
        off = cs + (16 if istcp else 6)
        assert inb[off] == 0 and inb[off + 1] == 0


def test_ecn_quirk_tcp_treated_as_udp():
    # gso_type TCPV4|ECN: hdr_len from the TCP header (:55,:100-110) but
    # istcp == false (:151): udp->len written over seq bytes 4-5, checksum with
    # proto 17 at csum_offset 16.  SURVEY §8a A6 observed seq bytes 05c8 0064
    # for a 4 x 1460 super-buffer with seq0 = 100.
    pkt = pktbuild.build(False, True, bytes(4 * 1460), pktbuild.ipv4_addr("10.0.0.1"),
                         pktbuild.ipv4_addr("10.0.0.2"), seq=100, fill_l4=False)
    st, _, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=GSO_TCPV4 | GSO_ECN, gso_size=1460,
                               csum_start=20, csum_offset=16)
    assert st == 0 and res["segment_size"] == 1500 and len(out) == 4 * 1500
    for s in segments(bytes(out), 1500):
        assert s[24:28].hex() == "05c80064"
        assert textbook.l4_checksum_native(s, False, False, 20) == 0  # verifies as UDP


def test_udp_zero_checksum_not_remapped():
    # A UDP checksum computing to 0 is stored as 0, not 0xFFFF (:202-204).
    # Search a payload whose segment checksum is 0.
    base = pktbuild.build(False, False, bytes(8), bytes(4), bytes(4), fill_l4=False)
    for x in range(65536):
        pkt = bytearray(base)
        pkt[28:30] = struct.pack(">H", x)
        st, _, out, _, res = split(bytes(pkt), flags=NEEDS_CSUM, gso_type=GSO_UDP_L4, gso_size=100, csum_start=20,
                                   csum_offset=6)
        if out[26] == 0 and out[27] == 0:
            assert textbook.l4_checksum_native(bytes(out), False, False, 20) in (0, 0xFFFF)
            return
    pytest.fail("no zero-checksum payload found")


def test_error_and_passthrough_cases():
    pkt = pktbuild.make_tcp(False, "192.0.2.1", 1, "192.0.2.2", 1, 0x18, 200, 9999)
    # gso_size 0 with payload: reference loops forever -> -1
    assert split(pkt, flags=NEEDS_CSUM, gso_type=GSO_TCPV4, gso_size=0, csum_start=20, csum_offset=16)[0] == -1
    # capacity below reserve_size -> -2
    st, *_ = oracle.gso_split(np.frombuffer(pkt, np.uint8), dict(flags=1, gso_type=1, gso_size=100, csum_start=20,
                                                                 csum_offset=16), 279)
    assert st == -2
    # unknown gso type (UFO = 3) -> passthrough untouched
    st, inb, out, _, res = split(pkt, flags=NEEDS_CSUM, gso_type=3, gso_size=100, csum_start=20, csum_offset=16)
    assert st == 0 and res["passthrough"] == 1 and bytes(inb) == pkt
    # TCP with a too-short L4 part -> passthrough
    st, _, _, _, res = split(pkt[:30], flags=NEEDS_CSUM, gso_type=GSO_TCPV4, gso_size=100, csum_start=20,
                             csum_offset=16)
    assert st == 0 and res["passthrough"] == 1
    # doff < 5 -> passthrough
    bad = bytearray(pkt)
    bad[32] = 0x40
    st, _, _, _, res = split(bytes(bad), flags=NEEDS_CSUM, gso_type=GSO_TCPV4, gso_size=100, csum_start=20,
                             csum_offset=16)
    assert st == 0 and res["passthrough"] == 1
    # GSO_NONE without NEEDS_CSUM: untouched
    st, inb, _, _, res = split(pkt, flags=0, gso_type=GSO_NONE, gso_size=100, csum_start=20, csum_offset=16)
    assert st == 0 and bytes(inb) == pkt and res["passthrough"] == 1
    # out of contract: csum_start inside the IPv4 header
    assert split(pkt, flags=NEEDS_CSUM, gso_type=GSO_UDP_L4, gso_size=100, csum_start=12, csum_offset=6)[0] == -3
    # empty payload: zero segments, prefix still zeroed
    st, inb, out, _, res = split(pkt[:40], flags=NEEDS_CSUM, gso_type=GSO_TCPV4, gso_size=100, csum_start=20,
                                 csum_offset=16)
    assert st == 0 and res["passthrough"] == 0 and res["out_len"] == 0 and inb[36] == 0 and inb[37] == 0


def test_batch_driver_matches_per_buffer():
    """orc_gso_split_desc (the threaded CPU baseline of config 3) gives the
    per-super-buffer oracle's bytes, statuses and in-place input changes."""
    rng = np.random.default_rng(31)
    pkts, vnets = [], []
    for k in range(40):
        isv6, istcp = bool(k & 1), bool(k & 2)
        p = pktbuild.build(isv6, istcp, rng.integers(0, 256, int(rng.integers(0, 9000)), dtype=np.uint8).tobytes(),
                           rng.integers(0, 256, 16 if isv6 else 4, dtype=np.uint8).tobytes(),
                           rng.integers(0, 256, 16 if isv6 else 4, dtype=np.uint8).tobytes(), fill_l4=False)
        gt = (4 if isv6 else 1) if istcp else 5
        vnets.append(dict(flags=1, gso_type=gt if k % 7 else 0, hdr_len=0, gso_size=int(rng.choice([100, 1448, 1460])),
                          csum_start=40 if isv6 else 20, csum_offset=16 if istcp else 6))
        pkts.append(p)
    d = np.zeros(len(pkts), dtype=oracle.GSO_DESC)
    io = oo = 0
    for k, (p, v) in enumerate(zip(pkts, vnets)):
        cap = len(p) + (len(p) // v["gso_size"] + 2) * 80
        d[k]["in_offset"], d[k]["out_offset"], d[k]["in_len"], d[k]["out_cap"] = io + 3, oo + 5, len(p), cap
        for f, x in v.items():
            d[k]["vnet"][f] = x
        io += len(p) + 3
        oo += cap + 5
    inbuf = np.zeros(io + 8, np.uint8)
    for k, p in enumerate(pkts):
        inbuf[int(d[k]["in_offset"]):int(d[k]["in_offset"]) + len(p)] = np.frombuffer(p, np.uint8)
    outbuf = np.zeros(oo + 8, np.uint8)
    before = inbuf.copy()
    st = oracle.gso_split_desc(inbuf, d, outbuf, threads=4)
    for k, (p, v) in enumerate(zip(pkts, vnets)):
        s1, in_after, out1, _, res = oracle.gso_split(np.frombuffer(p, np.uint8), v, int(d[k]["out_cap"]))
        assert int(st[k]) == s1
        o = int(d[k]["in_offset"])
        assert np.array_equal(inbuf[o:o + len(p)], in_after)
        if s1 == 0 and not res["passthrough"]:
            oo = int(d[k]["out_offset"])
            assert np.array_equal(outbuf[oo:oo + len(out1)], out1)
    assert not np.array_equal(before, inbuf)  # the reference zeroes prefix fields in place
