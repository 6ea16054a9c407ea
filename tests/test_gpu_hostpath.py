"""Host-memory encap and decap steps (SURVEY §8 f3 composed with A6, f1 and
f4): wg_encap_host (tun reads -> do_tun_gso_split -> Peer::encrypt per
segment, worker/encap.cpp:22-170) and wg_decap_host (UDP GRO batch ->
Peer::decrypt -> evaluate_packet, worker/decap.cpp:90-156,
worker/decap_ref.cpp:37-107), each against the oracle message for message:
odd totals, more chunks than the pipeline's three device slots
(host_chunk_mb = 1), pageable and pinned buffers (downloads into pinned
memory by the store kernel or the runtime's copy, knob host_d2h; misaligned
pinned outputs fall back to the copy), two host threads at once."""
import threading

import numpy as np
import pytest

import oracle
import pktbuild
from test_gpu_gso import random_case

pytestmark = pytest.mark.gpu


def _wga():
    import wireglider_amd as wga

    return wga


@pytest.fixture
def d2h():
    """Sets knob host_d2h for one test, restored after."""
    wga = _wga()
    saved = wga.tune_get("host_d2h")
    yield lambda v: wga.tune_set("host_d2h", v)
    wga.tune_set("host_d2h", saved)


@pytest.fixture
def small_chunks():
    wga = _wga()
    saved = wga.tune_get("host_chunk_mb")
    wga.tune_set("host_chunk_mb", 1)
    yield
    wga.tune_set("host_chunk_mb", saved)


MAX_SEG, MAX_SIZE = 48, 3000
MSG_CAP = MAX_SEG * (32 + (MAX_SIZE + 15) // 16 * 16)


def encap_case(seed, n=300):
    wga = _wga()
    rng = np.random.default_rng(seed)
    cases = [random_case(rng) for _ in range(n)]
    # config-3-shaped tun reads (64 KiB TCP super-buffers, 1,460-B segments)
    for k in range(60):
        p = pktbuild.build(False, True, rng.integers(0, 256, 65495, dtype=np.uint8).tobytes(),
                           pktbuild.ipv4_addr("10.0.0.1"), pktbuild.ipv4_addr("10.0.0.2"), seq=k * 7919,
                           fill_l4=False)
        cases.insert(int(rng.integers(0, len(cases))), (p, dict(flags=1, gso_type=1, gso_size=1460, csum_start=20,
                                                                 csum_offset=16), 73216))
    desc = np.zeros(len(cases), dtype=wga.GSO_DESC_DTYPE)
    off, caps = int(rng.integers(0, 17)), []
    for k, (pkt, vnet, cap) in enumerate(cases):
        if cap is None:
            cap = len(pkt) + (len(pkt) // max(1, vnet.get("gso_size", 1)) + 2) * 200
        caps.append(cap)
        desc[k]["in_offset"], desc[k]["in_len"], desc[k]["out_cap"] = off, len(pkt), cap
        for f in ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset"):
            desc[k]["vnet"][f] = vnet.get(f, 0)
        off += len(pkt) + int(rng.integers(0, 17))
    inbuf = np.zeros(off + 7, np.uint8)
    for k, (pkt, _, _) in enumerate(cases):
        o = int(desc[k]["in_offset"])
        inbuf[o:o + len(pkt)] = np.frombuffer(pkt, np.uint8)
    return cases, caps, desc, inbuf


def check_encap(cases, caps, key, rx, c0, msgs, res, gres, nxt):
    ctr = c0
    for i, (pkt, vnet, _) in enumerate(cases):
        st, o_in, o_out, _, r = oracle.gso_split(np.frombuffer(pkt, np.uint8), vnet, caps[i])
        assert int(gres[i]["status"]) == st, i
        S, ol = int(r["segment_size"]), int(r["out_len"])
        ns = nb = 0
        if st == 0 and S and ol:
            ns = (ol + S - 1) // S
            last = ol - (ns - 1) * S
            nb = (ns - 1) * (32 + (S + 15) // 16 * 16) + 32 + (last + 15) // 16 * 16
            if ns > MAX_SEG or S > MAX_SIZE or nb > MSG_CAP:
                ns = nb = 0
        assert (int(res[i]["nmsg"]), int(res[i]["msg_bytes"])) == (ns, nb), i
        if ns:
            assert int(res[i]["counter0"]) == ctr, i
            src = o_in if r["passthrough"] else o_out
            exp = oracle.wg_encrypt_batch(key, rx, ctr, src[:ol], S)
            np.testing.assert_array_equal(msgs[i * MSG_CAP:i * MSG_CAP + nb], exp, err_msg=f"super-buffer {i}")
        ctr += ns
    assert nxt == ctr and ctr - c0 > 300


@pytest.mark.parametrize("parts", [1, 3])
def test_encap_host_matches_oracle(gpu, small_chunks, parts):
    wga = _wga()
    cases, caps, desc, inbuf = encap_case(21)
    assert inbuf.size > 4 << 20  # more 1-MiB chunks than device slots
    key = bytes(range(1, 33))
    c0 = (1 << 32) - 100  # counters cross 2^32 on the way
    saved = wga.tune_get("encap_parts")
    wga.tune_set("encap_parts", parts)  # each chunk's device step pipelined in slices too
    try:
        msgs, res, gres, nxt = wga.encap_host(inbuf, desc, key, 0xABCD, c0, MAX_SEG, MAX_SIZE, MSG_CAP)
    finally:
        wga.tune_set("encap_parts", saved)
    check_encap(cases, caps, key, 0xABCD, c0, msgs, res, gres, nxt)


@pytest.mark.parametrize("mode", [0, 1])
def test_encap_host_pinned_two_threads(gpu, small_chunks, d2h, mode):
    """Two host threads, each with its own pipeline, concurrently; one of them
    reads its tun reads from and writes its messages to pinned buffers (by
    the store kernel when host_d2h = 1)."""
    wga = _wga()
    d2h(mode)
    work = [encap_case(31), encap_case(32)]
    key = bytes(32)
    out = [None, None]
    pins = []

    def run(k):
        cases, caps, desc, inbuf = work[k]
        if k == 1:
            pin_in, pin_out = wga.PinnedBuffer(inbuf.size), wga.PinnedBuffer(len(cases) * MSG_CAP)
            pins.extend([pin_in, pin_out])
            pin_in.array[:] = inbuf
            inbuf, msgs = pin_in.array, pin_out.array
        else:
            msgs = None
        for _ in range(2):
            out[k] = wga.encap_host(inbuf, desc, key, 7 + k, 1000 * k, MAX_SEG, MAX_SIZE, MSG_CAP, msgs=msgs)
        wga.host_release()

    ts = [threading.Thread(target=run, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in (0, 1):
        cases, caps, _, _ = work[k]
        msgs, res, gres, nxt = out[k]
        check_encap(cases, caps, key, 7 + k, 1000 * k, msgs, res, gres, nxt)
    for p in pins:
        p.close()


def test_encap_host_pinned_misaligned(gpu, small_chunks, d2h):
    """Pinned messages buffer 8 bytes off a 16-B boundary: the store kernel
    is skipped (runtime copy), the bytes around the region stay untouched."""
    wga = _wga()
    d2h(1)
    cases, caps, desc, inbuf = encap_case(33, n=120)
    need = len(cases) * MSG_CAP
    pin = wga.PinnedBuffer(need + 32)
    pin.array[:] = 0x5A
    key = bytes(range(32))
    msgs, res, gres, nxt = wga.encap_host(inbuf, desc, key, 3, 0, MAX_SEG, MAX_SIZE, MSG_CAP,
                                          msgs=pin.array[8:8 + need])
    check_encap(cases, caps, key, 3, 0, msgs, res, gres, nxt)
    assert (pin.array[:8] == 0x5A).all() and (pin.array[8 + need:] == 0x5A).all()
    pin.close()


def test_encap_host_empty_and_invalid(gpu):
    wga = _wga()
    d = np.zeros(0, dtype=wga.GSO_DESC_DTYPE)
    msgs, res, gres, nxt = wga.encap_host(np.zeros(16, np.uint8), d, bytes(32), 1, 55, 4, 100, 4 * 144)
    assert nxt == 55 and res.size == 0
    d = np.zeros(2, dtype=wga.GSO_DESC_DTYPE)
    d["in_offset"], d["in_len"] = [100, 0], 50  # out of input order: refused
    with pytest.raises(wga.WireGliderError):
        wga.encap_host(np.zeros(256, np.uint8), d, bytes(32), 1, 0, 4, 100, 4 * 144)
    with pytest.raises(wga.WireGliderError):  # msg_cap not a multiple of 16
        wga.encap_host(np.zeros(256, np.uint8), d[:1], bytes(32), 1, 0, 4, 100, 4 * 144 + 8)


def decap_case(seed, n, S=1504, short=700):
    """n data messages of S-byte plaintexts (S a multiple of 16, so decap's
    padded plaintext is the IP packet and the gates run), valid IPv4/IPv6 x
    TCP/UDP packets with stored checksums; some tampered (ciphertext, tag,
    counter past RejectAfterMessages, corrupted inner packet), the last one
    short by `short` bytes (an odd total)."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    pts = []
    for i in range(n):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        hl = (40 if v6 else 20) + (20 if tcp else 8)
        al = 16 if v6 else 4
        p = bytearray(pktbuild.build(v6, tcp, rng.integers(0, 256, S - hl, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                     rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        if rng.integers(0, 12) == 0:
            p[int(rng.integers(0, S))] ^= 0x40  # inner packet corrupted: gates fail
        pts.append(bytes(p))
    plain = np.frombuffer(b"".join(pts), np.uint8)[: n * S - short]
    msgs = oracle.wg_encrypt_batch(key, 0x77, 5000, plain, S).copy()
    stride = S + 32
    for i in rng.choice(n - 1, size=n // 20, replace=False):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            msgs[i * stride + 16 + int(rng.integers(0, S))] ^= 1  # ciphertext
        elif kind == 1:
            msgs[i * stride + stride - 1] ^= 0x80  # tag
        else:
            msgs[i * stride + 8:i * stride + 16] = 0xFF  # counter > RejectAfterMessages
    return key, msgs, stride


def check_decap(key, msgs, stride, got):
    plain, st, ver, l4 = got
    exp_plain, exp_st = oracle.wg_decrypt_batch(key, msgs, stride)
    np.testing.assert_array_equal(st, exp_st)
    n = exp_st.size
    ps = stride - 32
    ok = np.nonzero(exp_st == 0)[0]
    pv, gv = exp_plain.reshape(-1), plain.reshape(-1)
    for i in ok:
        ln = min(ps, msgs.size - i * stride - 32)
        np.testing.assert_array_equal(gv[i * ps:i * ps + ln], pv[i * ps:i * ps + ln], err_msg=f"message {i}")
    if ver is None:
        return
    d = np.zeros(n, dtype=oracle.PKT_DESC)
    d["offset"] = np.arange(n, dtype=np.uint64) * ps
    d["len"] = [min(ps, msgs.size - i * stride - 32) for i in range(n)]
    ev, el4 = oracle.verify_desc(exp_plain, d)
    ev[exp_st != 0], el4[exp_st != 0] = 0, 0
    np.testing.assert_array_equal(ver, ev)
    np.testing.assert_array_equal(l4, el4)
    assert (ev & 3 == 3).mean() > 0.7 and (exp_st != 0).sum() > 10


@pytest.mark.parametrize("verify", [True, False], ids=["decrypt+verify", "decrypt"])
def test_decap_host_matches_oracle(gpu, small_chunks, verify):
    wga = _wga()
    key, msgs, stride = decap_case(41, 3001)
    assert msgs.size > 4 << 20  # more 1-MiB chunks than device slots
    got = wga.decap_host(msgs, stride, key, verify=verify)
    check_decap(key, msgs, stride, got)


@pytest.mark.parametrize("mode", [0, 1, 3, 5])
def test_decap_host_pinned_two_threads(gpu, small_chunks, d2h, mode):
    """Two threads; one decrypts from and into pinned buffers.  Plaintext by
    the store kernel when host_d2h has bit 2 (3: every chunk) or bit 4 (5, the
    default: chunks under 24 MiB, all of them here); by the runtime's copy
    with neither (0, 1) — ADVICE r05: bit 2 was overridden for small chunks."""
    wga = _wga()
    d2h(mode)
    work = [decap_case(51, 2503, short=1), decap_case(52, 1999, S=1456, short=33)]
    out = [None, None]
    pins = []

    def run(k):
        key, msgs, stride = work[k]
        plain = None
        if k == 0:
            pin_m, pin_p = wga.PinnedBuffer(msgs.size), wga.PinnedBuffer((msgs.size // stride + 1) * (stride - 32))
            pins.extend([pin_m, pin_p])
            pin_m.array[:] = msgs
            msgs, plain = pin_m.array, pin_p.array
        for _ in range(2):
            out[k] = wga.decap_host(msgs, stride, key, plain=plain)
        wga.host_release()

    ts = [threading.Thread(target=run, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in (0, 1):
        check_decap(*work[k], out[k])
    for p in pins:
        p.close()


@pytest.mark.gpu
def test_host_path_keeps_current_device(gpu):
    """The host-memory entries and wg_host_release set the pipeline's device
    for their own scope and restore the caller's current device (ADVICE r02:
    release() had left it switched)."""
    import torch

    wga = _wga()
    before = torch.cuda.current_device()
    buf = bytes(np.random.default_rng(5).integers(0, 256, 1500 * 64, dtype=np.uint8))
    wga.calc_l4_checksum_host(buf, 1500, False, False, 20)
    assert torch.cuda.current_device() == before
    wga.host_release()
    assert torch.cuda.current_device() == before
    wga.calc_l4_checksum_host(buf, 1500, False, False, 20)  # the pipeline rebuilt after a release
    wga.host_release()
    assert torch.cuda.current_device() == before


@pytest.mark.gpu
def test_pipeline_build_failure(gpu):
    """A pipeline whose build fails part-way (the third event creation, forced
    by the WG_INTERNAL_TEST_FAULT_INJECT_PIPE hook, as under resource exhaustion) returns an
    error and leaves nothing half-built: the thread's next call builds the
    pipeline again and its results are bit-exact (a failed build
    had left the device marked, so later calls ran with null streams and
    events).  In a child process, since the hook is read once per process."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    code = (
        "import sys, numpy as np\n"
        f"sys.path[:0] = [{str(root)!r}, {str(root / 'oracle')!r}]\n"
        "import wireglider_amd as wga, oracle\n"
        "buf = np.random.default_rng(5).integers(0, 256, 1500 * 300, dtype=np.uint8)\n"
        "try:\n"
        "    wga.calc_l4_checksum_host(buf.tobytes(), 1500, False, False, 20)\n"
        "    print('FIRST ok')\n"
        "except wga.WireGliderError as e:\n"
        "    print('FIRST failed:', e)\n"
        "out = wga.calc_l4_checksum_host(buf.tobytes(), 1500, False, False, 20)\n"
        "print('SECOND', bool(np.array_equal(out, oracle.l4_uniform(buf, 1500, 20, 0))))\n")
    env = dict(os.environ, WG_INTERNAL_TEST_FAULT_INJECT_PIPE="3")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "FIRST failed" in r.stdout and "HIP runtime failure" in r.stdout, r.stdout
    assert "SECOND True" in r.stdout, r.stdout


@pytest.mark.gpu
def test_encap_host_small_reads_large_msg_cap(gpu, small_chunks):
    """Many ACK-sized tun reads with a msg_cap sized for 64-KiB TSO reads
    (ADVICE r03): chunks close on their output bytes too (messages at msg_cap
    each within twice the chunk budget), so the slots stay small; every
    message still matches the oracle, counters consecutive across chunks."""
    wga = _wga()
    rng = np.random.default_rng(33)
    cases = []
    for k in range(3000):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        p = pktbuild.build(v6, tcp, rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes(),
                           rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8).tobytes(),
                           rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8).tobytes(), fill_l4=False)
        cases.append((p, dict(flags=1, gso_type=0, csum_start=40 if v6 else 20, csum_offset=16 if tcp else 6), 4096))
    desc = np.zeros(len(cases), dtype=wga.GSO_DESC_DTYPE)
    off, caps = 5, []
    for k, (pkt, vnet, cap) in enumerate(cases):
        caps.append(cap)
        desc[k]["in_offset"], desc[k]["in_len"], desc[k]["out_cap"] = off, len(pkt), cap
        for f in ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset"):
            desc[k]["vnet"][f] = vnet.get(f, 0)
        off += len(pkt) + int(rng.integers(0, 9))
    inbuf = np.zeros(off + 7, np.uint8)
    for k, (pkt, _, _) in enumerate(cases):
        inbuf[int(desc[k]["in_offset"]):int(desc[k]["in_offset"]) + len(pkt)] = np.frombuffer(pkt, np.uint8)
    assert len(cases) * MSG_CAP > 2 * (2 << 20)  # the messages alone span many 2-MiB output budgets
    key = bytes(range(7, 39))
    msgs, res, gres, nxt = wga.encap_host(inbuf, desc, key, 0x77, 5, MAX_SEG, MAX_SIZE, MSG_CAP)
    ctr = 5
    for i, (pkt, vnet, _) in enumerate(cases):
        st, o_in, o_out, _, r = oracle.gso_split(np.frombuffer(pkt, np.uint8), vnet, caps[i])
        assert int(gres[i]["status"]) == st == 0, i
        ol, S = int(r["out_len"]), int(r["segment_size"])
        nb = 32 + (ol + 15) // 16 * 16
        assert (int(res[i]["nmsg"]), int(res[i]["msg_bytes"]), int(res[i]["counter0"])) == (1, nb, ctr), i
        src = o_in if r["passthrough"] else o_out
        np.testing.assert_array_equal(msgs[i * MSG_CAP:i * MSG_CAP + nb], oracle.wg_encrypt_batch(key, 0x77, ctr,
                                                                                                  src[:ol], S))
        ctr += 1
    assert nxt == ctr
