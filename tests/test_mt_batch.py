"""Several host threads on the batch entry points at once (SURVEY §8(b)
"Threading": the reference runs one worker thread per tun queue,
wireglider.cpp:117-151, each calling the checksum path for its own batches,
worker/offload.cpp:202, include/worker/evaluator.hpp:64,93).

tests/cpp/mt_batch.cpp (built by build()) drives the C ABI from 1-16
threads; this file writes its inputs and the oracle's expected outputs and
reads its JSON.  Conformance: every call's outputs are refilled with a
sentinel on the calling stream first and compared byte for byte with the
oracle after it, for wg_verify_desc, wg_l4csum_desc, wg_l4csum_uniform,
wg_gso_split, wg_checksum_desc, wg_verify_uniform and wg_aead_encrypt_batch,
with the threads on

  * their own streams;
  * hipStreamPerThread — one handle value that is a different stream in each
    thread (wg_verify_desc's per-stream state was keyed
    by the raw handle, so these threads shared entry lists and counters);
  * the legacy NULL stream (one stream shared by every thread);
  * a fresh stream per call, destroyed right after its launch (the next
    stream gets the same handle value).

`verify_small` 6 forces the compacting path on every call that has state;
the default (7) reaches it on runs of mixed batches.
"""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
import test_gpu_gso as tg
import test_verify_gates as tv

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "tests" / "cpp" / "bin" / "mt_batch"


def _sized(rng, n, lo, hi):
    pkts = []
    for _ in range(n):
        v6, tcp = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
        hl = (40 if v6 else 20) + (20 if tcp else 8)
        al = 16 if v6 else 4
        plen = int(rng.integers(max(0, lo - hl), max(1, hi - hl)))
        p = bytearray(tv.pktbuild.build(v6, tcp, rng.integers(0, 256, plen, dtype=np.uint8).tobytes(),
                                        rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                        rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        if rng.integers(0, 8) == 0:
            p[int(rng.integers(0, len(p)))] ^= 1 << int(rng.integers(0, 8))
        pkts.append(bytes(p))
    return pkts


def write_inputs(d: Path, seed: int = 61, n: int = 3000) -> dict:
    """The harness's inputs and the oracle's outputs as raw files in d."""
    rng = np.random.default_rng(seed)
    kinds = {"small": _sized(rng, n, 20, 65), "long": _sized(rng, n, 65, 1600),
             "mixed": tv.interleaved_batch(rng, n + 1)}
    stats = {}
    for k, pkts in kinds.items():
        buf, desc = tv.pack(pkts, rng)
        v, l4 = oracle.verify_desc(buf, desc)
        buf.tofile(d / f"verify_{k}.buf")
        desc.tofile(d / f"verify_{k}.desc")
        v.astype(np.uint8).tofile(d / f"verify_{k}.verdict")
        l4.astype(np.uint16).tofile(d / f"verify_{k}.l4")
        stats[k] = {"packets": len(pkts), "verified_ok": float(np.mean((v & tv.OK) == tv.OK))}
    # descriptor L4 batch: the mixed packets with per-packet csum_start / flags
    buf, desc = tv.pack(_sized(rng, 4000, 40, 9000), rng)
    desc["flags"] = rng.integers(0, 4, desc.size)
    desc["csum_start"] = np.minimum(desc["len"], np.where(desc["flags"] & 1, 40, 20))
    buf.tofile(d / "l4d.buf")
    desc.tofile(d / "l4d.desc")
    oracle.l4_desc(buf, desc).tofile(d / "l4d.out")
    oracle.checksum_desc(buf, desc).tofile(d / "l4d.plain")
    # uniform PacketBatch: 2,000 valid 1,500-B packets of every family, the
    # last one cut to 800 B (a short last segment), every 9th corrupted
    segs = []
    for i in range(2000):
        v6, tcp = bool(i & 1), bool(i & 2)
        hl, al = (40 if v6 else 20) + (20 if tcp else 8), 16 if v6 else 4
        p = bytearray(tv.pktbuild.build(v6, tcp, rng.integers(0, 256, 1500 - hl, dtype=np.uint8).tobytes(),
                                        rng.integers(0, 256, al, dtype=np.uint8).tobytes(),
                                        rng.integers(0, 256, al, dtype=np.uint8).tobytes()))
        if i % 9 == 0:
            p[int(rng.integers(0, 1500))] ^= 0x10
        segs.append(bytes(p))
    ubuf = np.frombuffer(b"".join(segs), np.uint8)[: 2000 * 1500 - 700].copy()
    ubuf.tofile(d / "l4u.buf")
    oracle.l4_uniform(ubuf, 1500, 20, 2).tofile(d / "l4u.out")
    ud = np.zeros(2000, dtype=oracle.PKT_DESC)
    ud["offset"] = np.arange(2000) * 1500
    ud["len"] = [min(1500, ubuf.size - 1500 * i) for i in range(2000)]
    uv, ul4 = oracle.verify_desc(ubuf, ud)
    uv.astype(np.uint8).tofile(d / "l4u.verdict")
    ul4.astype(np.uint16).tofile(d / "l4u.l4")
    key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    rx, c0 = 0x1234567, (1 << 33) + 5
    (d / "aead.key").write_bytes(key)
    oracle.wg_encrypt_batch(key, rx, c0, ubuf, 1500).tofile(d / "aead.out")
    (d / "params.txt").write_text(f"1500 20 2 {rx} {c0}\n")
    stats["uniform_verified_ok"] = float(np.mean((uv & tv.OK) == tv.OK))
    # GSO: random super-buffers the oracle splits with status 0
    cases = []
    while len(cases) < 48:
        pkt, vnet, _ = tg.random_case(rng)
        if len(pkt) > 20000 or vnet["gso_size"] == 0:
            continue
        cap = len(pkt) + (len(pkt) // max(1, vnet["gso_size"]) + 2) * 200
        if oracle.gso_split(np.frombuffer(pkt, np.uint8), vnet, cap)[0] == 0:
            cases.append((pkt, vnet, cap))
    gd = np.zeros(len(cases), dtype=oracle.GSO_DESC)
    io = oo = 0
    for k, (pkt, vnet, cap) in enumerate(cases):
        io += int(rng.integers(0, 17))
        oo += int(rng.integers(0, 17))
        gd[k]["in_offset"], gd[k]["out_offset"], gd[k]["in_len"], gd[k]["out_cap"] = io, oo, len(pkt), cap
        for f in ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset"):
            gd[k]["vnet"][f] = vnet.get(f, 0)
        io += len(pkt)
        oo += cap
    gin = np.zeros(io + 64, np.uint8)
    for k, (pkt, _, _) in enumerate(cases):
        gin[int(gd[k]["in_offset"]): int(gd[k]["in_offset"]) + len(pkt)] = np.frombuffer(pkt, np.uint8)
    gin.tofile(d / "gso.in")
    gd.tofile(d / "gso.desc")
    after = gin.copy()
    gout = np.full(oo + 64, 0xA5, np.uint8)  # the harness refills with the same sentinel
    st = oracle.gso_split_desc(after, gd, gout)
    assert np.all(st == 0)
    gout.tofile(d / "gso.out")
    after.tofile(d / "gso.in_after")
    st.astype(np.int8).tofile(d / "gso.status")
    stats["gso_super_buffers"] = len(cases)
    return stats


def run_harness(d: Path, *args, env_extra=None, timeout=240) -> dict:
    assert EXE.exists(), f"{EXE} not built (build() builds it)"
    env = dict(os.environ)
    env.update(env_extra or {})
    r = subprocess.run([str(EXE), str(d), *map(str, args)], capture_output=True, text=True, timeout=timeout,
                       env=env)
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_inputs_match_oracle_self_consistency(tmp_path):
    """CPU: the input writer itself (the oracle's outputs, the GSO cases all
    status 0, the verify kinds really small / long / mixed)."""
    st = write_inputs(tmp_path, n=400)
    assert st["gso_super_buffers"] == 48
    v = np.fromfile(tmp_path / "verify_small.desc", dtype=oracle.PKT_DESC)
    assert v["len"].max() <= 64
    v = np.fromfile(tmp_path / "verify_long.desc", dtype=oracle.PKT_DESC)
    assert v["len"].min() > 64
    v = np.fromfile(tmp_path / "verify_mixed.desc", dtype=oracle.PKT_DESC)
    assert (v["len"] <= 64).any() and (v["len"] > 64).any()
    assert st["long"]["verified_ok"] > 0.5
    assert 0.5 < st["uniform_verified_ok"] < 1.0
    assert (tmp_path / "aead.out").stat().st_size == 1999 * 1536 + 32 + 800


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    d = tmp_path_factory.mktemp("mt_batch")
    write_inputs(d)
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("verify_small", [7, 6])
@pytest.mark.parametrize("stream", ["perthread", "own", "legacy"])
def test_mt_conformance(gpu, inputs, stream, verify_small):
    """4 threads x 50 iterations x seven entry points, every call's outputs
    equal the oracle's."""
    res = run_harness(inputs, "conform", 4, 50, stream, env_extra={"WG_VERIFY_SMALL": str(verify_small)})
    print(json.dumps(res))
    assert res["errors"] == 0 and res["mismatched"] == 0, res
    assert res["ops"]["wg_verify_desc"]["calls"] == 200


@pytest.mark.gpu
@pytest.mark.parametrize("verify_small", [7, 6])
def test_mt_stream_churn(gpu, inputs, verify_small):
    """4 threads, each verifying 50 mixed / small / long batches on a fresh
    stream per call, destroyed right after the launch (hipStreamDestroy waits
    for the pending work, profiles/r06_stream_identity.txt): the next stream
    gets the same handle value and inherits its state; every call's verdicts
    and L4 results equal the oracle's."""
    res = run_harness(inputs, "conform", 4, 50, "churn", env_extra={"WG_VERIFY_SMALL": str(verify_small)})
    print(json.dumps(res))
    assert res["errors"] == 0 and res["mismatched"] == 0, res


@pytest.mark.gpu
def test_mt_sixteen_threads(gpu, inputs):
    """16 threads on their own streams (one per tun queue of a 16-queue
    device), 20 iterations each."""
    res = run_harness(inputs, "conform", 16, 20, "own")
    print(json.dumps(res))
    assert res["errors"] == 0 and res["mismatched"] == 0, res


@pytest.mark.gpu
def test_mt_one_thread(gpu, inputs):
    """The same conformance run with one thread (the 1-thread point of the
    launch-rate figure)."""
    res = run_harness(inputs, "conform", 1, 50, "own")
    print(json.dumps(res))
    assert res["errors"] == 0 and res["mismatched"] == 0, res
