"""Parity of the gfx950 data-message AEAD (wireglider_amd/csrc/aead.hip)
with the oracle (oracle/aead_oracle.c, pinned by RFC 8439 and OpenSSL
vectors in tests/test_oracle_aead.py), through the C ABI.

Encrypt: Peer::encrypt for every segment of a PacketBatch (proto/proto.cpp:
544-583, worker/encap.cpp:136-141) — byte-identical messages, at every
segment size class the kernel distinguishes (every power-of-two group size,
64-lane groups in several passes up to 64 KiB, under each aead_k blocking),
short last segments, empty
segments (keepalives), counters across 2^32 and RejectAfterMessages.
Decrypt: Peer::decrypt for every message of a GRO batch (proto.cpp:496-523) —
plaintexts, statuses, zeroed output on a bad tag, untouched output on the
pre-MAC rejections.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
G = json.loads((Path(__file__).resolve().parent / "golden" / "aead" / "aead_golden.json").read_text())


def _wga():
    import wireglider_amd as wga

    return wga


def _dev(a, gpu):
    import torch

    return torch.from_numpy(np.array(a, dtype=np.uint8, copy=True)).to(gpu)


ENC_CASES = [(1460, 1460 * 40 + 777), (1460, 1460 * 3), (64, 64 * 300 + 1), (1, 17), (15, 15 * 9 + 4), (16, 16 * 33),
             (17, 17 * 20 + 16), (1984, 1984 * 10 + 5), (1985, 1985 * 9 + 1984), (4032, 4032 * 4 + 63),
             (4033, 4033 * 3 + 1), (9000, 9000 * 5 + 8999), (65535, 65535 * 2 + 100), (1500, 1500 * 64),
             # one-pass limits of the 64-lane group at K = 2 / 4 (127 / 255 payload blocks) and past them
             (8128, 8128 * 3 + 1), (8129, 8129 * 2 + 8128), (16320, 16320 * 2 + 5), (16321, 16321 * 2 + 16000),
             (32768, 32768 * 2 + 1)]


@pytest.fixture(params=[(0, 1), (2, 1), (3, 1), (0, 0), (2, 0)], ids=lambda kp: f"aead_k={kp[0]},stage={kp[1]}")
def aead_k(request):
    """Every lane-blocking variant (consecutive ChaCha20 blocks per lane: 2,
    3 or chosen per batch) with encrypt's messages staged in LDS or stored
    from the lanes: speed knobs that must not change any byte."""
    wga = _wga()
    saved = {k: wga.tune_get(k) for k in ("aead_k", "aead_stage")}
    wga.tune_set("aead_k", request.param[0])
    wga.tune_set("aead_stage", request.param[1])
    yield request.param
    for k, v in saved.items():
        wga.tune_set(k, v)


@pytest.mark.parametrize("seg,total", ENC_CASES)
def test_encrypt_batch_matches_oracle(gpu, aead_k, seg, total):
    import torch

    wga = _wga()
    rng = np.random.default_rng(seg * 7 + total)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    counter0 = int(rng.choice([0, 5, (1 << 32) - 3, (1 << 63) + 11]))
    exp = oracle.wg_encrypt_batch(key, 0xC0FFEE, counter0, buf, seg)
    out, st = wga.aead_encrypt_batch(_dev(buf, gpu), seg, key, 0xC0FFEE, counter0)
    torch.cuda.synchronize()
    got = out.cpu().numpy()[: exp.size]
    n = (total + seg - 1) // seg
    assert (st.cpu().numpy()[:n] == 0).all()
    stride = wga.aead_message_stride(seg)
    for i in range(n):  # compare message by message: the first mismatch names its packet
        a, b = i * stride, min((i + 1) * stride, exp.size)
        assert np.array_equal(got[a:b], exp[a:b]), f"message {i} of {n} (seg {seg})"


def test_encrypt_golden_wireguard_vectors(gpu):
    """OpenSSL-generated WireGuard messages (tests/golden/aead), one-packet batches."""
    import torch

    wga = _wga()
    for k, v in enumerate(G["wg"]):
        pt = np.frombuffer(bytes.fromhex(v["pt"]), np.uint8)
        if pt.size == 0:
            continue  # an empty PacketBatch has no segment (keepalives: test_keepalive_and_rejections)
        out, st = wga.aead_encrypt_batch(_dev(pt.copy(), gpu), pt.size, bytes.fromhex(v["key"]), k, v["counter"])
        torch.cuda.synchronize()
        if v["counter"] >= oracle.REJECT_AFTER_MESSAGES:  # proto.cpp:560-562 refuses before encrypting
            assert int(st.cpu()[0]) == -1
            continue
        assert int(st.cpu()[0]) == 0
        msg = out.cpu().numpy().tobytes()
        assert msg[:16] == (4).to_bytes(4, "little") + k.to_bytes(4, "little") + v["counter"].to_bytes(8, "little")
        assert msg[16:-16].hex() == v["ct"] and msg[-16:].hex() == v["tag"]


def test_counter_rejections_and_wrap(gpu):
    import torch

    wga = _wga()
    key = bytes(range(32))
    buf = np.arange(100 * 10, dtype=np.uint8)
    c0 = oracle.REJECT_AFTER_MESSAGES - 4  # packets 4.. hit counter >= RejectAfterMessages
    out = torch.full((wga.aead_message_stride(100) * 10,), 0xAB, dtype=torch.uint8, device=gpu)
    out, st = wga.aead_encrypt_batch(_dev(buf, gpu), 100, key, 9, c0, out=out)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    assert list(s) == [0] * 4 + [-1] * 6
    exp = oracle.wg_encrypt_batch(key, 9, c0, buf[:400], 100)
    got = out.cpu().numpy()
    assert np.array_equal(got[: exp.size], exp)
    assert (got[exp.size:] == 0xAB).all()  # rejected packets write nothing


def _messages(rng, key, seg_pt, n, counter0=1):
    buf = rng.integers(0, 256, seg_pt * n, dtype=np.uint8)
    return oracle.wg_encrypt_batch(key, 3, counter0, buf, seg_pt), buf


@pytest.mark.parametrize("seg_pt", [1, 16, 63, 1440, 1460, 1984, 2000, 4032, 4100, 9000, 16320, 40000])
def test_decrypt_batch_matches_oracle(gpu, aead_k, seg_pt):
    import torch

    wga = _wga()
    rng = np.random.default_rng(seg_pt)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    n = 40 if seg_pt < 5000 else 12
    if seg_pt > 10000:
        n = 10
    msgs, _ = _messages(rng, key, seg_pt, n)
    mseg = wga.aead_message_stride(seg_pt)
    msgs = msgs.copy()
    # tamper: ciphertext bit, tag bit, counter (nonce) bit, and a truncated last message
    msgs[2 * mseg + 16 + (seg_pt // 2)] ^= 0x10
    msgs[5 * mseg + mseg - 1] ^= 0x01
    msgs[7 * mseg + 9] ^= 0x40
    msgs[9 * mseg + 8: 9 * mseg + 16] = np.frombuffer((oracle.REJECT_AFTER_MESSAGES + 1).to_bytes(8, "little"), np.uint8)
    for trunc in (0, 5, mseg - 20, mseg - 31):
        m = msgs[: msgs.size - trunc] if trunc else msgs
        exp_pt, exp_st = oracle.wg_decrypt_batch(key, m, mseg)
        out = torch.full((max(exp_pt.size, 1),), 0xEE, dtype=torch.uint8, device=gpu)
        pt, st = wga.aead_decrypt_batch(_dev(m, gpu), mseg, key, out=out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(st.cpu().numpy()[: exp_st.size], exp_st, err_msg=f"trunc {trunc}")
        np.testing.assert_array_equal(pt.cpu().numpy()[: exp_pt.size], exp_pt, err_msg=f"trunc {trunc}")
        assert exp_st[2] == exp_st[5] == exp_st[7] == exp_st[9] == -1 and exp_st[0] == 0


def test_keepalive_and_rejections(gpu, aead_k):
    """32-byte keepalives (encrypt of an empty payload, worker/encap.cpp:156)
    decrypt to nothing; 15- and 31-byte messages are rejected untouched."""
    import torch

    wga = _wga()
    key = bytes(range(100, 132))
    ka = b"".join(oracle.wg_encrypt(key, 1, c, b"") for c in range(50))
    pt, st = wga.aead_decrypt_batch(_dev(np.frombuffer(ka, np.uint8), gpu), 32, key)
    torch.cuda.synchronize()
    assert (st.cpu().numpy()[:50] == 0).all()
    for ln in (15, 31):
        m = np.frombuffer(ka[:ln], np.uint8)
        out = torch.full((32,), 0xEE, dtype=torch.uint8, device=gpu)
        pt, st = wga.aead_decrypt_batch(_dev(m, gpu), 64, key, out=out)
        torch.cuda.synchronize()
        assert int(st.cpu()[0]) == -1
        assert (pt.cpu().numpy() == 0xEE).all()  # rejected before the MAC: untouched


def test_round_trip_on_device(gpu, aead_k):
    """GPU encrypt -> GPU decrypt of a config-3-shaped batch (45 segments of
    1460 B and a 1295-B last one, the GSO output the encap worker encrypts)."""
    import torch

    wga = _wga()
    rng = np.random.default_rng(3)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pts = rng.integers(0, 256, 1460 * 44 + 1295, dtype=np.uint8)
    out, st = wga.aead_encrypt_batch(_dev(pts, gpu), 1460, key, 77, 1000)
    mseg = wga.aead_message_stride(1460)
    pt, st2 = wga.aead_decrypt_batch(out, mseg, key)
    torch.cuda.synchronize()
    assert (st2.cpu().numpy() == 0).all()
    p = pt.cpu().numpy().reshape(-1)
    for i in range(45):
        ln = 1460 if i < 44 else 1295
        assert np.array_equal(p[i * (mseg - 32): i * (mseg - 32) + ln], pts[i * 1460: i * 1460 + ln])


@pytest.mark.parametrize("seg_pt", [1504, 1500, 9008, 64, 48, 20])
def test_decrypt_verify_matches_oracle(gpu, aead_k, seg_pt):
    """Decrypt + the decap verify gates in one pass (wg_aead_decrypt_verify_batch)
    == the oracle's decrypt, then the oracle's evaluate_packet gates over each
    plaintext at its libsodium (padded) length, as worker/decap_ref.cpp:81-86
    hands it to push_packet: a 1,504-B packet (a multiple of 16) passes the IP
    gates, a 1,500-B one cannot (its padded length is not its ip_len).  Mixed
    v4/v6 x TCP/UDP with valid checksums, one corrupted payload byte, one
    corrupted header byte, one bad tag, one rejected counter."""
    import torch

    wga = _wga()
    rng = np.random.default_rng(seg_pt + 17)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    n = 120
    buf = torch.empty(n * seg_pt, dtype=torch.uint8, device=gpu)
    wga.synth_fill(buf, seg_pt)
    desc = wga.synth_desc_stride(n, seg_pt, seg_pt, 1, seg_pt, 0, device=gpu)
    wga.synth_headers(buf, desc, seg_pt, 0)
    if seg_pt >= 48:
        wga.store_l4csum(buf, desc, wga.calc_l4_checksum_desc(buf, desc))
    torch.cuda.synchronize()
    pts = buf.cpu().numpy().copy()
    pts[3 * seg_pt + seg_pt - 1] ^= 0x20  # payload byte: L4 checksum fails
    pts[5 * seg_pt + 13] ^= 0x01  # a v4 source-address byte (IP checksum) / v6 address byte (L4 checksum)
    msgs = oracle.wg_encrypt_batch(key, 3, 77, pts, seg_pt).copy()
    mseg = wga.aead_message_stride(seg_pt)
    msgs[7 * mseg + mseg - 2] ^= 0x04  # tag
    msgs[9 * mseg + 8: 9 * mseg + 16] = np.frombuffer((oracle.REJECT_AFTER_MESSAGES + 1).to_bytes(8, "little"), np.uint8)
    exp_pt, exp_st = oracle.wg_decrypt_batch(key, msgs, mseg)
    out, st, ver, l4 = wga.aead_decrypt_verify_batch(_dev(msgs, gpu), mseg, key)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st.cpu().numpy()[:n], exp_st)
    plen = mseg - 32
    got_pt = out.cpu().numpy()[: n * plen]
    ok = exp_st == 0
    for i in np.nonzero(ok)[0]:
        assert np.array_equal(got_pt[i * plen:(i + 1) * plen], exp_pt[i * plen:(i + 1) * plen]), i
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = np.arange(n, dtype=np.uint64) * plen
    d["len"] = plen
    ev, el4 = oracle.verify_desc(exp_pt, d)
    ev[~ok], el4[~ok] = 0, 0
    np.testing.assert_array_equal(ver.cpu().numpy()[:n], ev)
    np.testing.assert_array_equal(l4.cpu().numpy()[:n], el4)
    if seg_pt == 1504:  # the gates really ran: most packets pass both, the corrupted ones do not
        assert np.count_nonzero(ev & 0x03 == 0x03) >= n - 4 and ev[3] & 0x02 == 0
