"""The encap worker's step on the device (wg_encap_encrypt, SURVEY §8 f4 on
A6's output): every segment of wg_gso_split's PacketBatches encrypted for one
peer with consecutive counters in super-buffer / segment order, as
worker/encap.cpp:136-141 runs Peer::encrypt per segment with
encrypt_nonce++ — compared message for message with the oracle's
wg_encrypt_batch over each PacketBatch (the GSO output itself is pinned in
tests/test_gpu_gso.py).  Random super-buffers of every GSO type: splits,
passthrough (GSO_NONE, unknown types), errors (no messages), batches past
the segment / size / capacity bounds (no messages).

fused=True runs the same step through wg_encap_batch (the headers-only split
+ the AEAD reading payload from the input): its messages, counters, result
records, GSO results and input prefix zeroing must equal the two-call path's,
and the segment headers it leaves in `out` the split's.  With encap_synth=1
the AEAD builds the headers (fields, IPv4 and L4 checksums) of the
super-buffers it encrypts whose header fits one 64-B block, and the split
skips those: the same comparisons pin every synthesized header byte and the
messages encrypted over it."""
import numpy as np
import pytest

import oracle
from test_gpu_gso import random_case

pytestmark = pytest.mark.gpu


def _wga():
    import wireglider_amd as wga

    return wga


@pytest.mark.parametrize("fused", [False, True], ids=["split+encrypt", "encap_batch"])
@pytest.mark.parametrize("seed", [11, 12])
@pytest.mark.parametrize("knobs", [{}, {"aead_k": 2}, {"aead_k": 3}, {"aead_stage": 0}, {"encap_parts": 2},
                                   {"encap_parts": 3}, {"encap_parts": 8}, {"encap_spw": 4}, {"encap_spw": 0},
                                   {"aead_k": 2, "encap_parts": 2}, {"encap_synth": 1},
                                   {"encap_synth": 1, "aead_k": 2}, {"encap_synth": 1, "encap_parts": 3},
                                   {"encap_synth": 1, "aead_stage": 0}, {"encap_synth": 0}],
                         ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()) or "default")
def test_encap_matches_oracle(gpu, seed, knobs, fused):
    import torch

    wga = _wga()
    saved = {k: wga.tune_get(k) for k in knobs}
    for k, v in knobs.items():
        wga.tune_set(k, v)
    rng = np.random.default_rng(seed)
    cases = [random_case(rng) for _ in range(250)]
    n = len(cases)
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    in_off = out_off = 0
    for k, (pkt, vnet, cap) in enumerate(cases):
        in_off += int(rng.integers(0, 17))
        out_off += int(rng.integers(0, 17))
        if cap is None:
            cap = len(pkt) + (len(pkt) // max(1, vnet.get("gso_size", 1)) + 2) * 200
        desc[k]["in_offset"], desc[k]["out_offset"] = in_off, out_off
        desc[k]["in_len"], desc[k]["out_cap"] = len(pkt), cap
        for f in ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset"):
            desc[k]["vnet"][f] = vnet.get(f, 0)
        in_off += len(pkt)
        out_off += cap
    inbuf = np.zeros(in_off + 64, np.uint8)
    for k, (pkt, _, _) in enumerate(cases):
        o = int(desc[k]["in_offset"])
        inbuf[o:o + len(pkt)] = np.frombuffer(pkt, np.uint8)
    d_in = torch.from_numpy(inbuf).to(gpu)
    d_out = torch.zeros(out_off + 64, dtype=torch.uint8, device=gpu)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    d_in_f = d_in.clone()  # the fused call's own copy (the split zeroes prefix fields in place)
    d_res = wga.gso_split(d_in, d_desc, d_out)
    max_seg, max_size, cap = 48, 9100, 48 * (32 + 9104)
    if "encap_synth" in knobs:
        # header synthesis runs with the staged AEAD (segments up to ~6 KB):
        # super-buffers of larger segments get no messages and keep the split
        max_size = 1600
    cap_small = 7000  # some super-buffers' messages will not fit: nmsg 0
    msg_off = np.arange(n, dtype=np.int64) * cap
    msgs = torch.full((n * cap + 64,), 0xEE, dtype=torch.uint8, device=gpu)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    c0 = int(rng.choice([1, (1 << 32) - 40]))
    m_cap = cap_small if seed == 12 else cap
    d_msg_off = torch.from_numpy(msg_off).to(gpu)
    if fused:
        d_hdr = torch.full_like(d_out, 0x5A)
        d_res_f = torch.zeros_like(d_res)
        eres, total = wga.encap_batch(d_in_f, d_desc, d_hdr, d_res_f, key, 0xBEEF, c0, d_msg_off, m_cap, max_seg,
                                      max_size, msgs)
    else:
        eres, total = wga.encap_encrypt(d_in, d_out, d_desc, d_res, key, 0xBEEF, c0, d_msg_off, m_cap, max_seg,
                                        max_size, msgs)
    torch.cuda.synchronize()
    for k, v in saved.items():
        wga.tune_set(k, v)
    g_in, g_out = d_in.cpu().numpy(), d_out.cpu().numpy()
    r = d_res.cpu().numpy().view(wga.GSO_RESULT_DTYPE)
    e = eres.cpu().numpy().view(wga.ENCAP_RESULT_DTYPE)
    got = msgs.cpu().numpy()
    if fused:
        assert torch.equal(d_res_f, d_res)
        assert torch.equal(d_in_f, d_in)
        g_hdr = d_hdr.cpu().numpy()
        for i in range(n):
            if int(r[i]["status"]) or int(r[i]["passthrough"]):
                continue
            S, ol, hl = int(r[i]["segment_size"]), int(r[i]["out_len"]), int(r[i]["hdr_len"])
            o = int(desc[i]["out_offset"])
            for so in range(0, ol, S):
                np.testing.assert_array_equal(g_hdr[o + so:o + so + hl], g_out[o + so:o + so + hl],
                                              err_msg=f"super-buffer {i} segment header at {so}")
    ctr, n_msgs = c0, 0
    for i in range(n):
        S, ol = int(r[i]["segment_size"]), int(r[i]["out_len"])
        ns = nb = 0
        if int(r[i]["status"]) == 0 and S and ol:
            ns = (ol + S - 1) // S
            last = ol - (ns - 1) * S
            nb = (ns - 1) * (32 + (S + 15) // 16 * 16) + 32 + (last + 15) // 16 * 16
            if ns > max_seg or S > max_size or nb > m_cap:
                ns = nb = 0
        assert (int(e[i]["nmsg"]), int(e[i]["msg_bytes"])) == (ns, nb), i
        if ns:
            assert int(e[i]["counter0"]) == ctr, i
            src = (g_in[int(desc[i]["in_offset"]):] if int(r[i]["passthrough"]) else g_out[int(desc[i]["out_offset"]):])
            exp = oracle.wg_encrypt_batch(key, 0xBEEF, ctr, src[:ol], S)
            o = int(msg_off[i])
            assert exp.size == nb
            np.testing.assert_array_equal(got[o:o + nb], exp, err_msg=f"super-buffer {i}")
            assert np.all(got[o + nb:o + min(m_cap, cap)] == 0xEE), i  # nothing past its messages
        else:
            assert np.all(got[int(msg_off[i]):int(msg_off[i]) + 64] == 0xEE), i
        ctr += ns
        n_msgs += ns
    assert int(total.cpu()[0]) == n_msgs and n_msgs > 50


@pytest.mark.parametrize("fused,synth", [(False, 0), (True, 0), (True, 1)],
                         ids=["split+encrypt", "encap_batch", "encap_batch-synth"])
def test_encap_reject_after_messages(gpu, fused, synth):
    """Counters crossing RejectAfterMessages inside a super-buffer: the
    reference's encrypt refuses every counter >= it (proto.cpp:560-562) but
    still advances encrypt_nonce, and the encap worker advances its outbuf
    over accepted messages only (worker/encap.cpp:138-140): super-buffer 0 is
    all accepted, super-buffer 1 keeps its first 2 messages, super-buffer 2
    none; nmsg / counter0 / the total count every segment.  Refused segments
    still get their headers (synth: built and checksummed by the AEAD)."""
    import torch

    import pktbuild

    wga = _wga()
    n, gso, pay = 3, 100, 500  # 5 segments each
    pkts = [pktbuild.make_tcp(False, "192.0.2.1", 1, "192.0.2.2", 1, 0x18, pay, 1000 + k) for k in range(n)]
    cap = 8192
    desc = np.zeros(n, dtype=wga.GSO_DESC_DTYPE)
    desc["in_offset"] = np.arange(n) * 1024
    desc["out_offset"] = np.arange(n) * cap
    desc["in_len"], desc["out_cap"] = [len(p) for p in pkts], cap
    for f, v in (("flags", 1), ("gso_type", 1), ("hdr_len", 40), ("gso_size", gso), ("csum_start", 20),
                 ("csum_offset", 16)):
        desc["vnet"][f] = v
    inbuf = np.zeros(n * 1024, np.uint8)
    for k, p in enumerate(pkts):
        inbuf[k * 1024:k * 1024 + len(p)] = np.frombuffer(p, np.uint8)
    d_in = torch.from_numpy(inbuf).to(gpu)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    d_out = torch.zeros(n * cap, dtype=torch.uint8, device=gpu)
    key = bytes(range(32))
    c0 = oracle.REJECT_AFTER_MESSAGES - 7  # super-buffer 1's segments 2-4 are refused
    msg_off = torch.from_numpy(np.arange(n, dtype=np.int64) * cap).to(gpu)
    msgs = torch.full((n * cap,), 0xEE, dtype=torch.uint8, device=gpu)
    d_res = wga.gso_split(d_in.clone(), d_desc, d_out)
    if fused:
        saved = wga.tune_get("encap_synth")
        wga.tune_set("encap_synth", synth)
        d_hdr = torch.zeros_like(d_out)
        try:
            eres, total = wga.encap_batch(d_in.clone(), d_desc, d_hdr, torch.zeros_like(d_res), key, 7, c0, msg_off,
                                          cap, 8, 200, msgs)
            torch.cuda.synchronize()
        finally:
            wga.tune_set("encap_synth", saved)
        g_hdr, g_seg = d_hdr.cpu().numpy(), d_out.cpu().numpy()
        for i in range(n):
            for so in range(0, 5 * 140, 140):
                o = i * cap + so
                np.testing.assert_array_equal(g_hdr[o:o + 40], g_seg[o:o + 40], err_msg=f"{i} {so}")
    else:
        eres, total = wga.encap_encrypt(d_in, d_out, d_desc, d_res, key, 7, c0, msg_off, cap, 8, 200, msgs)
    torch.cuda.synchronize()
    e = eres.cpu().numpy().view(wga.ENCAP_RESULT_DTYPE)
    got, segs = msgs.cpu().numpy(), d_out.cpu().numpy()
    stride = 32 + (140 + 15) // 16 * 16
    assert int(total.cpu()[0]) == 5 * n
    assert list(e["nmsg"]) == [5, 5, 5]
    assert list(e["counter0"]) == [c0, c0 + 5, c0 + 10]
    assert list(e["msg_bytes"]) == [5 * stride, 2 * stride, 0]
    for i, keep in enumerate((5, 2, 0)):
        ol = 5 * 140
        exp = oracle.wg_encrypt_batch(key, 7, c0 + 5 * i, segs[i * cap:i * cap + ol], 140)
        np.testing.assert_array_equal(got[i * cap:i * cap + keep * stride], exp[:keep * stride])
        assert np.all(got[i * cap + keep * stride:(i + 1) * cap] == 0xEE), i  # refused messages: nothing written
