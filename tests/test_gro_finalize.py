"""GRO finalize: oracle restatement pinned by an independent
RFC textbook, and GPU parity of wg_gro_finalize.

Reference semantics: PacketRefBatch::finalize (include/worker/flowkey_ref.hpp:82-117)
and OwnedPacketBatch::finalize (include/worker/flowkey_own.hpp:83-115).  The
reference's tests hold no finalize vectors, so the restatement is pinned by
the textbook (tests/textbook.py): after finalize, the header's lengths are the
coalesced packet's, its IPv4 header checksum verifies, and the NEEDS_CSUM seed
is the complemented pseudo-header sum over the header's addresses.  The
reference's own call sums std::span objects (pointer-dependent)
and is deliberately not reproduced.
"""
import struct

import numpy as np
import pytest

import oracle
import pktbuild
import textbook


def _flow(rng, isv6, istcp, payload_len, opts=b""):
    al = 16 if isv6 else 4
    src = rng.integers(0, 256, al, dtype=np.uint8).tobytes()
    dst = rng.integers(0, 256, al, dtype=np.uint8).tobytes()
    payload = rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()
    pkt = pktbuild.build(isv6, istcp, payload, src, dst, 7, 9, 1234, ip_options=b"" if isv6 else opts)
    cs = (40 if isv6 else 20 + len(opts))
    hdr_len = cs + (20 if istcp else 8)
    return pkt, cs, hdr_len


def _expected(pkt, cs, hdr_len, isv6, istcp):
    """Textbook: the coalesced packet's header with lengths as built, IPv4
    checksum verifying, L4 field = ~pseudo-header sum (native order)."""
    h = bytearray(pkt[:hdr_len])
    l4len = len(pkt) - cs
    if isv6:
        pseudo = h[8:24] + h[24:40] + struct.pack(">I", l4len & 0xFFFF) + b"\x00\x00\x00" + bytes([h[6]])
    else:
        pseudo = h[12:16] + h[16:20] + b"\x00" + bytes([h[9]]) + struct.pack(">H", l4len & 0xFFFF)
    seed = textbook.bswap16(textbook.rfc_checksum_be(bytes(pseudo)))
    off = cs + (16 if istcp else 6)
    h[off:off + 2] = struct.pack("<H", seed)
    return bytes(h)


@pytest.mark.parametrize("isv6", [False, True])
@pytest.mark.parametrize("istcp", [False, True])
def test_oracle_gro_finalize_textbook(isv6, istcp):
    rng = np.random.default_rng(100 + 2 * isv6 + istcp)
    for payload_len in (0, 1, 17, 1448, 64000):
        for opts in (b"", b"\x01\x01\x01\x00", bytes(40)):
            pkt, cs, hdr_len = _flow(rng, isv6, istcp, payload_len, opts)
            want = _expected(pkt, cs, hdr_len, isv6, istcp)
            # stale header as GRO holds it: lengths of the first segment, junk sums
            stale = bytearray(pkt[:hdr_len])
            stale[2:4] = b"\x12\x34"
            if not isv6:
                stale[10:12] = b"\xde\xad"
            else:
                stale[4:6] = b"\x00\x10"
            if not istcp:
                stale[cs + 4:cs + 6] = b"\x00\x09"
            off = cs + (16 if istcp else 6)
            stale[off:off + 2] = b"\xbe\xef"
            if isv6:
                stale[2:4] = pkt[2:4]
            st, got = oracle.gro_finalize(np.frombuffer(bytes(stale), np.uint8), cs, off - cs, isv6, istcp,
                                          payload_len)
            assert st == 0
            assert got.tobytes() == want, (isv6, istcp, payload_len, len(opts))
            if not isv6:
                assert oracle.checksum(got[:cs]) == 0


def test_oracle_gro_finalize_l4len_truncates():
    """l4len is passed as uint16 to the length fields and the pseudo-header
    (flowkey_ref.hpp:84-86,95,108-112): a >64 KiB coalesced flow wraps."""
    rng = np.random.default_rng(5)
    pkt, cs, hdr_len = _flow(rng, False, False, 100)
    st, got = oracle.gro_finalize(np.frombuffer(pkt[:hdr_len], np.uint8), cs, 6, False, False, 70000)
    assert st == 0
    l4len = hdr_len - cs + 70000
    assert struct.unpack(">H", got[cs + 4:cs + 6].tobytes())[0] == l4len & 0xFFFF
    assert struct.unpack(">H", got[2:4].tobytes())[0] == (hdr_len + 70000) & 0xFFFF


@pytest.mark.parametrize("cs,off,hdr_len,isv6,istcp", [
    (19, 16, 40, False, True),   # csum_start inside the IPv4 header
    (20, 16, 30, False, True),   # field past the header
    (40, 6, 47, True, False),    # UDP header truncated
    (41, 16, 40, True, True),    # csum_start past the header
])
def test_oracle_gro_finalize_out_of_contract(cs, off, hdr_len, isv6, istcp):
    h = np.arange(hdr_len, dtype=np.uint8)
    st, got = oracle.gro_finalize(h, cs, off, isv6, istcp, 10)
    assert st == -3 and np.array_equal(got, h)


def _batch(rng, n):
    """A ragged batch of flow headers (v4/v6, TCP/UDP, IPv4 options,
    payloads up to and past 64 KiB) plus some out-of-contract descriptors."""
    import wireglider_amd as wg

    hdrs, desc = bytearray(), np.zeros(n, dtype=wg.GRO_DESC_DTYPE)
    for i in range(n):
        isv6, istcp = bool(rng.integers(2)), bool(rng.integers(2))
        opts = bytes(4 * int(rng.integers(0, 11))) if not isv6 else b""
        pkt, cs, hdr_len = _flow(rng, isv6, istcp, int(rng.integers(0, 64)), opts)
        h = bytearray(rng.integers(0, 256, hdr_len, dtype=np.uint8).tobytes())
        h[:cs] = pkt[:cs]  # keep version/proto/addresses; everything else junk
        off = 16 if istcp else 6
        if i % 13 == 7:  # csum_start well past the IP header (> 64 B: the kernel's general path)
            extra = int(rng.integers(20, 60))
            h = h[:cs] + bytearray(rng.integers(0, 256, extra, dtype=np.uint8).tobytes()) + h[cs:]
            cs, hdr_len = cs + extra, hdr_len + extra
        if i % 17 == 5:
            cs = int(rng.integers(0, 20))  # out of contract
        pad = int(rng.integers(0, 8))
        hdrs += bytes(pad)
        desc[i] = (len(hdrs), int(rng.integers(0, 90000)), hdr_len, cs, off,
                   (1 if isv6 else 0) | (2 if istcp else 0), 0x55)
        hdrs += h
    return np.frombuffer(bytes(hdrs), np.uint8).copy(), desc


def _oracle_batch_per_flow(hdrs, desc):
    out, st = hdrs.copy(), np.zeros(len(desc), np.int8)
    for i, d in enumerate(desc):
        o, L = int(d["hdr_offset"]), int(d["hdr_len"])
        s, h = oracle.gro_finalize(out[o:o + L], int(d["csum_start"]), int(d["csum_offset"]), bool(d["flags"] & 1),
                                   bool(d["flags"] & 2), int(d["payload_bytes"]))
        out[o:o + L], st[i] = h, s
    return out, st


def test_oracle_gro_batch_matches_per_flow():
    pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    hdrs, desc = _batch(rng, 500)
    a, sa = _oracle_batch_per_flow(hdrs, desc)
    b, sb = oracle.gro_finalize_desc(hdrs, desc, threads=3)
    assert np.array_equal(a, b) and np.array_equal(sa, sb)


def _oracle_batch(hdrs, desc):
    return oracle.gro_finalize_desc(hdrs, desc)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2024, 2025])
def test_gpu_gro_finalize_parity(gpu, seed):
    import torch

    import wireglider_amd as wg

    rng = np.random.default_rng(seed)
    hdrs, desc = _batch(rng, 3000)
    want, want_st = _oracle_batch(hdrs, desc)
    assert (want_st == -3).any() and (want_st == 0).any()
    dh = torch.from_numpy(hdrs).to(gpu)
    dd = torch.from_numpy(desc.view(np.uint8)).to(gpu)
    wg.gro_finalize(dh, dd)
    torch.cuda.synchronize()
    got = dh.cpu().numpy()
    got_desc = dd.cpu().numpy().view(wg.GRO_DESC_DTYPE)
    assert np.array_equal(got_desc["status"], want_st)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_gro_finalize_empty(gpu):
    import torch

    import wireglider_amd as wg

    wg.gro_finalize(torch.zeros(0, dtype=torch.uint8, device=gpu), torch.zeros(0, dtype=torch.uint8, device=gpu))


@pytest.mark.gpu
def test_gpu_gro_finalize_high_addresses(gpu):
    """The same ragged batch placed so its flows straddle bit 31 and 4 GiB of
    a 4.3 GB header buffer (64-bit header offsets, staged-chunk addresses)."""
    import torch

    import wireglider_amd as wg

    rng = np.random.default_rng(2031)
    hdrs, desc = _batch(rng, 3000)
    want, want_st = _oracle_batch(hdrs, desc)
    big = torch.zeros((1 << 32) + (1 << 22), dtype=torch.uint8, device=gpu)
    for base in ((1 << 31) - hdrs.size // 2 + 3, (1 << 32) - hdrs.size // 2 + 9):
        d = desc.copy()
        d["hdr_offset"] += base
        big[base:base + hdrs.size] = torch.from_numpy(hdrs).to(gpu)
        dd = torch.from_numpy(d.view(np.uint8).copy()).to(gpu)
        wg.gro_finalize(big, dd)
        torch.cuda.synchronize()
        assert np.array_equal(dd.cpu().numpy().view(wg.GRO_DESC_DTYPE)["status"], want_st)
        assert np.array_equal(big[base:base + hdrs.size].cpu().numpy(), want)
    del big
    torch.cuda.empty_cache()
