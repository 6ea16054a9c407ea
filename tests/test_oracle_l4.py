"""Pin the oracle's calc_l4_checksum restatement (checksum.cpp:8-36).

checksum.cpp itself is unbuildable here (boost.endian and the un-vendored
fastcsum are absent), so the L4 path is pinned by (a) the reference test's
own assertion — a correctly checksummed packet verifies to 0 for v4/v6 x
TCP/UDP (tests/test-checksum.cpp:53-82); (b) flipped checksums must be
rejected (tests/test-flowkey-own.cpp:56-63,170-200 "coalesceItemInvalidCSum");
and (c) an independent RFC 768/793 textbook implementation (tests/textbook.py)
on random packets, odd lengths and odd csum_start.
"""
import struct

import numpy as np
import pytest

import oracle
import pktbuild
import textbook

FAMS = [(False, True), (False, False), (True, True), (True, False)]


@pytest.mark.parametrize("isv6,istcp", FAMS)
def test_l4_known_answer_verifies_to_zero(isv6, istcp):
    # tests/test-checksum.cpp:53-82: IP("192.0.2.2","192.0.2.1") / L4(1,1) /
    # RawPDU(create_packet(100)), calc_l4_checksum(pkt, ..., header_size) == 0.
    from pathlib import Path

    payload = np.fromfile(Path(__file__).parent / "golden" / "ref" / "create_packet_65536.bin",
                          dtype=np.uint8)[:100].tobytes()
    a = pktbuild.ipv6_addr if isv6 else pktbuild.ipv4_addr
    src, dst = ("2001:db8::1", "2001:db8::2") if isv6 else ("192.0.2.1", "192.0.2.2")
    pkt = pktbuild.build(isv6, istcp, payload, a(src), a(dst), 1, 1)
    cs = 40 if isv6 else 20
    assert oracle.calc_l4_checksum(pkt, isv6, istcp, cs) == 0


@pytest.mark.parametrize("isv6,istcp", FAMS)
def test_flipped_checksum_rejected(isv6, istcp):
    # flip_l4_csum (tests/test-flowkey-own.cpp:56-63) -> verify != 0
    rng = np.random.default_rng(7)
    pkt = bytearray(pktbuild.build(isv6, istcp, rng.integers(0, 256, 200, dtype=np.uint8).tobytes(),
                                   bytes(16 if isv6 else 4), bytes(range(16))[: 16 if isv6 else 4]))
    cs = 40 if isv6 else 20
    off = cs + (16 if istcp else 6)
    assert oracle.calc_l4_checksum(bytes(pkt), isv6, istcp, cs) == 0
    pkt[off] ^= 0xFF
    pkt[off + 1] ^= 0xFF
    assert oracle.calc_l4_checksum(bytes(pkt), isv6, istcp, cs) != 0


def test_l4_random_vs_textbook():
    rng = np.random.default_rng(0x5EED)
    for it in range(3000):
        isv6 = bool(rng.integers(0, 2))
        istcp = bool(rng.integers(0, 2))
        minlen = 40 if isv6 else 20
        n = int(rng.integers(minlen, 1600))
        pkt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        cs = int(rng.integers(0, n + 1))  # includes odd and == len
        got = oracle.calc_l4_checksum(pkt, isv6, istcp, cs)
        assert got == textbook.l4_checksum_native(pkt, isv6, istcp, cs), (it, n, cs)


@pytest.mark.parametrize("n", [64, 1500, 9000])
@pytest.mark.parametrize("isv6,istcp", FAMS)
def test_generate_then_verify(n, isv6, istcp):
    rng = np.random.default_rng(n)
    pkt = bytearray(pktbuild.random_packet(rng, isv6, istcp, n))
    cs = 40 if isv6 else 20
    c = oracle.calc_l4_checksum(bytes(pkt), isv6, istcp, cs)
    assert c == textbook.l4_checksum_native(bytes(pkt), isv6, istcp, cs)
    off = cs + (16 if istcp else 6)
    pkt[off:off + 2] = struct.pack("<H", c)  # native order store (offload.cpp:202-204)
    assert oracle.calc_l4_checksum(bytes(pkt), isv6, istcp, cs) == 0


def test_l4len_truncated_to_u16():
    # l4Len is uint16_t (include/netio/checksum.hpp:107): 65536 + 100 bytes of
    # L4 data carry length 100 in the pseudo-header.
    rng = np.random.default_rng(3)
    n = 20 + 65536 + 100
    pkt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    assert oracle.calc_l4_checksum(pkt, False, False, 20) == textbook.l4_checksum_native(pkt, False, False, 20)


def test_batched_drivers_match_scalar():
    rng = np.random.default_rng(11)
    seg, n = 1500, 257
    buf = rng.integers(0, 256, seg * n - 77, dtype=np.uint8)
    out = oracle.l4_uniform(buf, seg, 20, 0, threads=4)
    assert out.size == n
    for i in range(n):
        p = buf[i * seg:(i + 1) * seg]
        assert out[i] == oracle.calc_l4_checksum(p, False, False, 20)
    desc = np.zeros(n, dtype=oracle.PKT_DESC)
    desc["offset"] = np.arange(n) * seg
    desc["len"] = [min(seg, buf.size - i * seg) for i in range(n)]
    desc["csum_start"] = 40
    desc["flags"] = 3
    out2 = oracle.l4_desc(buf, desc, threads=3)
    for i in range(n):
        p = buf[int(desc["offset"][i]):int(desc["offset"][i]) + int(desc["len"][i])]
        assert out2[i] == oracle.calc_l4_checksum(p, True, True, 40)
