"""ctypes binding of the CPU oracle (oracle/csum_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
package wireglider_amd never imports this module.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libcsum_oracle.so"

PKT_DESC = np.dtype([("offset", "<u8"), ("len", "<u4"), ("csum_start", "<u2"), ("flags", "u1"),
                     ("reserved", "u1")])
assert PKT_DESC.itemsize == 16

VNET_HDR = np.dtype([("flags", "u1"), ("gso_type", "u1"), ("hdr_len", "<u2"), ("gso_size", "<u2"),
                     ("csum_start", "<u2"), ("csum_offset", "<u2")])
GSO_RESULT = np.dtype([("out_len", "<u8"), ("segment_size", "<u8"), ("hdr_len", "<u2"), ("isv6", "u1"),
                       ("ecn", "u1"), ("passthrough", "u1"), ("pad", "u1", 3)])
assert GSO_RESULT.itemsize == 24


class _VNet(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint8), ("gso_type", ctypes.c_uint8), ("hdr_len", ctypes.c_uint16),
                ("gso_size", ctypes.c_uint16), ("csum_start", ctypes.c_uint16), ("csum_offset", ctypes.c_uint16)]


class _GsoRes(ctypes.Structure):
    _fields_ = [("out_len", ctypes.c_uint64), ("segment_size", ctypes.c_uint64), ("hdr_len", ctypes.c_uint16),
                ("isv6", ctypes.c_uint8), ("ecn", ctypes.c_uint8), ("passthrough", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 3)]


def build() -> None:
    import subprocess

    subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)


def _load():
    if not LIB.exists():
        build()
    lib = ctypes.CDLL(str(LIB))
    vp, u64, u32, u16, i32, sz = (ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint16,
                                  ctypes.c_int, ctypes.c_size_t)
    lib.orc_checksum_ref1.restype = u16
    lib.orc_checksum_ref1.argtypes = [vp, sz]
    lib.orc_nofold.restype = u64
    lib.orc_nofold.argtypes = [vp, sz, u64]
    lib.orc_nofold_scalar.restype = u64
    lib.orc_nofold_scalar.argtypes = [vp, sz, u64]
    lib.orc_have_avx2.restype = i32
    lib.orc_have_avx2.argtypes = []
    lib.orc_fold_complement.restype = u16
    lib.orc_fold_complement.argtypes = [u64]
    lib.orc_checksum.restype = u16
    lib.orc_checksum.argtypes = [vp, sz, u64]
    lib.orc_pseudo_header_nofold.restype = u64
    lib.orc_pseudo_header_nofold.argtypes = [ctypes.c_uint8, vp, vp, sz, u16]
    lib.orc_calc_l4_checksum.restype = u16
    lib.orc_calc_l4_checksum.argtypes = [vp, sz, i32, i32, u16]
    lib.orc_l4_uniform.restype = None
    lib.orc_l4_uniform.argtypes = [vp, u64, u32, u16, u32, vp, i32]
    lib.orc_l4_desc.restype = None
    lib.orc_l4_desc.argtypes = [vp, vp, u64, vp, i32]
    lib.orc_checksum_desc.restype = None
    lib.orc_checksum_desc.argtypes = [vp, vp, u64, vp, i32]
    lib.orc_gso_split.restype = i32
    lib.orc_gso_split.argtypes = [vp, sz, ctypes.POINTER(_VNet), vp, sz, ctypes.POINTER(_GsoRes)]
    lib.orc_verify.restype = ctypes.c_uint8
    lib.orc_verify.argtypes = [vp, sz, vp]
    lib.orc_verify_desc.restype = None
    lib.orc_verify_desc.argtypes = [vp, vp, u64, vp, vp, i32]
    lib.orc_gro_finalize.restype = i32
    lib.orc_gro_finalize.argtypes = [vp, sz, u16, u16, i32, i32, u64]
    lib.orc_gro_finalize_desc.restype = None
    lib.orc_gro_finalize_desc.argtypes = [vp, vp, u64, i32]
    lib.orc_gso_split_desc.restype = None
    lib.orc_gso_split_desc.argtypes = [vp, vp, u64, vp, vp, i32]
    lib.orc_chacha20_block.restype = None
    lib.orc_chacha20_block.argtypes = [vp, u32, vp, vp]
    lib.orc_poly1305.restype = None
    lib.orc_poly1305.argtypes = [vp, vp, sz, vp]
    lib.orc_aead_encrypt.restype = None
    lib.orc_aead_encrypt.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp]
    lib.orc_aead_decrypt.restype = i32
    lib.orc_aead_decrypt.argtypes = [vp, vp, vp, sz, vp, sz, vp, vp]
    lib.orc_wg_encrypt.restype = sz
    lib.orc_wg_encrypt.argtypes = [vp, u32, u64, vp, sz, vp]
    lib.orc_wg_decrypt.restype = i32
    lib.orc_wg_decrypt.argtypes = [vp, vp, sz, vp]
    lib.orc_wg_encrypt_batch.restype = None
    lib.orc_wg_encrypt_batch.argtypes = [vp, u32, u64, vp, u64, u32, vp]
    lib.orc_wg_decrypt_batch.restype = None
    lib.orc_wg_decrypt_batch.argtypes = [vp, vp, u64, u32, vp, vp]
    lib.orc_wg_encrypt_batch_mt.restype = None
    lib.orc_wg_encrypt_batch_mt.argtypes = [vp, u32, u64, vp, u64, u32, vp, i32]
    lib.orc_wg_decrypt_batch_mt.restype = None
    lib.orc_wg_decrypt_batch_mt.argtypes = [vp, vp, u64, u32, vp, vp, i32]
    lib.orc_pool_stats_reset.restype = None
    lib.orc_pool_stats_reset.argtypes = []
    lib.orc_pool_stats.restype = i32
    lib.orc_pool_stats.argtypes = [vp, vp, i32]
    lib.orc_read_probe.restype = u64
    lib.orc_read_probe.argtypes = [vp, u64, i32]
    lib.orc_numa_retouch.restype = i32
    lib.orc_numa_retouch.argtypes = [vp, u64, i32]
    lib.orc_time_l4_uniform.restype = ctypes.c_double
    lib.orc_time_l4_uniform.argtypes = [vp, u64, u32, u16, u32, vp, i32, i32]
    return lib


lib = _load()


def _cgroup_cpu_quota() -> float | None:
    """CPUs granted by the cgroup CPU controller (v2 cpu.max or v1
    cfs_quota/period), or None when unlimited / not visible."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except Exception:
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else q / per
    except Exception:
        return None


def host_cores() -> dict:
    """The host cores this process may run on: the scheduler affinity mask
    (os.sched_getaffinity), capped by a cgroup CPU quota when one is set.
    `threads` is what the CPU baseline uses; the other fields say why."""
    import math

    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpu_quota()
    used = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"threads": used, "affinity": aff, "cgroup_quota_cpus": quota, "cpu_count": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def _cpu_busy(cpus: list, interval: float = 0.3) -> dict:
    """Busy fraction of each CPU in `cpus` over `interval` s (/proc/stat)."""
    import time

    def snap():
        out = {}
        for line in Path("/proc/stat").read_text().splitlines():
            if line.startswith("cpu") and line[3:4].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:9]]
                out[int(f[0][3:])] = (sum(v), v[3] + v[4])  # total, idle + iowait
        return out

    a = snap()
    time.sleep(interval)
    b = snap()
    res = {}
    for c in cpus:
        if c in a and c in b:
            dt = b[c][0] - a[c][0]
            res[c] = 1.0 - (b[c][1] - a[c][1]) / dt if dt > 0 else 1.0
    return res


def _core_of(c: int):
    base = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
    try:
        return (int((base / "physical_package_id").read_text()), int((base / "core_id").read_text()))
    except Exception:
        return (0, c)


def _l3_of(c: int) -> str:
    """The L3 domain of CPU c: the first CPU of its L3's shared_cpu_list
    (EPYC: one CCD), or "?" where sysfs does not say."""
    try:
        lst = Path(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read_text().strip()
        return lst.split(",")[0].split("-")[0]
    except Exception:
        return "?"


def _package_of(c: int) -> int:
    try:
        return int(Path(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id").read_text())
    except Exception:
        return 0


def quiet_cpus(n: int, policy: str = "spread") -> dict:
    """n CPUs of the affinity mask for n pinned workers, spread over the L3
    domains (CCDs): one physical core per worker, the domains dealt round
    robin (quietest domain first), the quietest CPUs first within a domain.
    A 16-worker leg then spans 16 CCDs instead of the 2-4 CCDs that the lowest
    CPU numbers of an idle host give (the all-core leg
    on CPUs 1-30, four CCDs, ran 3.2x one core).  Returns {"cpus": [...],
    "busy": mean busy fraction of the chosen CPUs before the run, "l3_domains":
    {domain: [cpus]} of the chosen CPUs}.

    policy "socket": the same dealing over the L3 domains of ONE package (the
    quietest that has n cores), so the workers share a socket's memory and
    coherence domain — what a library with process-wide atomics (OpenSSL 3's
    EVP layer) needs; bench.py times the all-core leg both ways and keeps the
    faster."""
    cpus = sorted(os.sched_getaffinity(0))
    busy = _cpu_busy(cpus)
    doms: dict = {}
    seen_cores = set()
    for c in sorted(cpus, key=lambda c: (busy.get(c, 1.0), c)):
        k = _core_of(c)
        if k in seen_cores:  # one CPU per physical core (SMT siblings left out)
            continue
        seen_cores.add(k)
        doms.setdefault(_l3_of(c), []).append(c)
    # the domains, quietest first (mean busy of their cores), then by number
    order = sorted(doms, key=lambda d: (sum(busy.get(c, 1.0) for c in doms[d]) / len(doms[d]),
                                        int(d) if d.isdigit() else 1 << 30))
    if policy == "socket":
        pk: dict = {}
        for d in order:
            pk.setdefault(_package_of(doms[d][0]), []).append(d)
        fits = [k for k, ds in pk.items() if sum(len(doms[d]) for d in ds) >= n]
        if fits:  # the quietest package that holds n workers
            best = min(fits, key=lambda k: sum(busy.get(c, 1.0) for d in pk[k] for c in doms[d])
                       / sum(len(doms[d]) for d in pk[k]))
            order = [d for d in order if d in pk[best]]
    chosen = []
    depth = 0
    while len(chosen) < n and any(depth < len(doms[d]) for d in order):
        for d in order:
            if depth < len(doms[d]) and len(chosen) < n:
                chosen.append(doms[d][depth])
        depth += 1
    for c in sorted(cpus, key=lambda c: (busy.get(c, 1.0), c)):  # fewer cores than n: SMT siblings
        if len(chosen) == n:
            break
        if c not in chosen:
            chosen.append(c)
    used: dict = {}
    for c in chosen:
        used.setdefault(_l3_of(c), []).append(c)
    return {"cpus": chosen, "busy": round(sum(busy.get(c, 1.0) for c in chosen) / max(1, len(chosen)), 4),
            "l3_domains": used, "policy": policy, "packages": sorted({_package_of(c) for c in chosen})}


def numa_of(c: int):
    """The NUMA node of CPU c (sysfs nodeN link), or None."""
    try:
        for e in Path(f"/sys/devices/system/cpu/cpu{c}").iterdir():
            if e.name.startswith("node") and e.name[4:].isdigit():
                return int(e.name[4:])
    except Exception:
        pass
    return None


def pool_stats_reset() -> None:
    lib.orc_pool_stats_reset()


def pool_stats(max_workers: int = 256) -> list:
    """[(busy_seconds, calls)] per worker of the persistent pool since the
    last reset."""
    busy = np.zeros(max_workers, np.uint64)
    calls = np.zeros(max_workers, np.uint64)
    n = int(lib.orc_pool_stats(busy.ctypes.data, calls.ctypes.data, max_workers))
    return [(float(busy[t]) * 1e-9, int(calls[t])) for t in range(n)]


def numa_retouch(buf, threads: int) -> bool:
    """Move buf's whole pages to the NUMA nodes of the pool's pinned workers
    (ORC_CPUS; page range t copied back by worker t after the range was
    dropped): contents unchanged.  False when it could not (buf left as is)."""
    a = np.asarray(buf)
    assert a.flags["C_CONTIGUOUS"] and a.flags["WRITEABLE"]
    return int(lib.orc_numa_retouch(a.ctypes.data, a.nbytes, threads)) == 0


def read_probe(buf, threads: int) -> int:
    """Read-only pass over buf's whole 4-KiB blocks by `threads` pinned
    workers (the CPU baseline's memory-path probe); returns the word sum."""
    a = _u8(buf)
    return int(lib.orc_read_probe(a.ctypes.data, a.size, threads))


def cgroup_throttling() -> dict | None:
    """cgroup v2 cpu.stat throttling counters (nr_throttled, throttled_usec),
    or None when not visible."""
    try:
        kv = dict(line.split() for line in Path("/sys/fs/cgroup/cpu.stat").read_text().splitlines())
        return {"nr_throttled": int(kv.get("nr_throttled", 0)), "throttled_usec": int(kv.get("throttled_usec", 0))}
    except Exception:
        return None


def default_threads() -> int:
    return host_cores()["threads"]


def _u8(buf) -> np.ndarray:
    a = np.ascontiguousarray(np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf)
    assert a.dtype == np.uint8
    return a


def checksum_ref1(buf) -> int:
    a = _u8(buf)
    return int(lib.orc_checksum_ref1(a.ctypes.data, a.size))


def checksum(buf, initial: int = 0) -> int:
    a = _u8(buf)
    return int(lib.orc_checksum(a.ctypes.data, a.size, initial))


def nofold(buf, initial: int = 0) -> int:
    a = _u8(buf)
    return int(lib.orc_nofold(a.ctypes.data, a.size, initial))


def nofold_scalar(buf, initial: int = 0) -> int:
    a = _u8(buf)
    return int(lib.orc_nofold_scalar(a.ctypes.data, a.size, initial))


def have_avx2() -> bool:
    return bool(lib.orc_have_avx2())


def fold_complement(x: int) -> int:
    return int(lib.orc_fold_complement(x))


def calc_l4_checksum(pkt, isv6: bool, istcp: bool, csum_start: int) -> int:
    a = _u8(pkt)
    return int(lib.orc_calc_l4_checksum(a.ctypes.data, a.size, int(isv6), int(istcp), csum_start))


def l4_uniform(buf: np.ndarray, segment_size: int, csum_start: int, flags: int,
               threads: int | None = None) -> np.ndarray:
    a = _u8(buf)
    n = (a.size + segment_size - 1) // segment_size
    out = np.empty(n, dtype=np.uint16)
    lib.orc_l4_uniform(a.ctypes.data, a.size, segment_size, csum_start, flags, out.ctypes.data,
                       threads or default_threads())
    return out


def l4_desc(buf: np.ndarray, desc: np.ndarray, threads: int | None = None) -> np.ndarray:
    a = _u8(buf)
    d = np.ascontiguousarray(desc).view(PKT_DESC).reshape(-1)
    out = np.empty(d.size, dtype=np.uint16)
    lib.orc_l4_desc(a.ctypes.data, d.ctypes.data, d.size, out.ctypes.data, threads or default_threads())
    return out


def checksum_desc(buf: np.ndarray, desc: np.ndarray, threads: int | None = None) -> np.ndarray:
    a = _u8(buf)
    d = np.ascontiguousarray(desc).view(PKT_DESC).reshape(-1)
    out = np.empty(d.size, dtype=np.uint16)
    lib.orc_checksum_desc(a.ctypes.data, d.ctypes.data, d.size, out.ctypes.data, threads or default_threads())
    return out


V_IP_OK, V_L4_OK, V_TCP, V_UDP, V_V6 = 0x01, 0x02, 0x04, 0x08, 0x10


def verify(pkt) -> tuple[int, int]:
    a = _u8(pkt)
    c = ctypes.c_uint16(0)
    v = int(lib.orc_verify(a.ctypes.data, a.size, ctypes.byref(c)))
    return v, int(c.value)


def verify_desc(buf: np.ndarray, desc: np.ndarray, threads: int | None = None):
    a = _u8(buf)
    d = np.ascontiguousarray(desc).view(PKT_DESC).reshape(-1)
    verdict = np.empty(d.size, dtype=np.uint8)
    l4 = np.empty(d.size, dtype=np.uint16)
    lib.orc_verify_desc(a.ctypes.data, d.ctypes.data, d.size, verdict.ctypes.data, l4.ctypes.data,
                        threads or default_threads())
    return verdict, l4


def gro_finalize(hdr, csum_start: int, csum_offset: int, isv6: bool, istcp: bool, payload_bytes: int):
    """Returns (status, header after)."""
    a = np.array(_u8(hdr), copy=True)
    st = int(lib.orc_gro_finalize(a.ctypes.data, a.size, csum_start, csum_offset, int(isv6), int(istcp),
                                  payload_bytes))
    return st, a


GRO_DESC = np.dtype([("hdr_offset", "<u8"), ("payload_bytes", "<u8"), ("hdr_len", "<u2"), ("csum_start", "<u2"),
                     ("csum_offset", "<u2"), ("flags", "u1"), ("status", "i1")])
assert GRO_DESC.itemsize == 24


def gro_finalize_desc(hdrs: np.ndarray, desc: np.ndarray, threads: int | None = None):
    """Batched GRO finalize; returns (headers after, status array).  Inputs
    are not modified."""
    a = np.array(_u8(hdrs), copy=True)
    d = np.array(np.ascontiguousarray(desc).view(GRO_DESC).reshape(-1), copy=True)
    end = (d["hdr_offset"].astype(np.int64) + d["hdr_len"]).max() if d.size else 0
    if end > a.size:
        raise ValueError("gro_finalize_desc: descriptor past the header buffer")
    lib.orc_gro_finalize_desc(a.ctypes.data, d.ctypes.data, d.size, threads or default_threads())
    return a, d["status"].copy()


def gro_working_copies(hdrs: np.ndarray, desc: np.ndarray):
    """Mutable copies of a GRO batch for gro_finalize_desc_inplace (made
    outside any timed region)."""
    return (np.array(_u8(hdrs), copy=True),
            np.array(np.ascontiguousarray(desc).view(GRO_DESC).reshape(-1), copy=True))


def gro_finalize_desc_inplace(hdrs: np.ndarray, desc: np.ndarray, threads: int | None = None) -> None:
    """Batched GRO finalize in place (headers and status), the C call only:
    the CPU baseline's timed leg."""
    assert hdrs.flags["C_CONTIGUOUS"] and desc.dtype == GRO_DESC and desc.flags["C_CONTIGUOUS"]
    lib.orc_gro_finalize_desc(hdrs.ctypes.data, desc.ctypes.data, desc.size, threads or default_threads())


def gso_split(inbuf: np.ndarray, vnet: dict, out_cap: int):
    """Returns (status, in_after, out_bytes, vnet_after, result dict)."""
    a = np.array(_u8(inbuf), copy=True)
    v = _VNet(vnet.get("flags", 0), vnet.get("gso_type", 0), vnet.get("hdr_len", 0), vnet.get("gso_size", 0),
              vnet.get("csum_start", 0), vnet.get("csum_offset", 0))
    out = np.zeros(max(out_cap, 1), dtype=np.uint8)
    r = _GsoRes()
    st = lib.orc_gso_split(a.ctypes.data, a.size, ctypes.byref(v), out.ctypes.data, out_cap, ctypes.byref(r))
    res = dict(out_len=r.out_len, segment_size=r.segment_size, hdr_len=r.hdr_len, isv6=r.isv6, ecn=r.ecn,
               passthrough=r.passthrough)
    vafter = dict(flags=v.flags, gso_type=v.gso_type, hdr_len=v.hdr_len, gso_size=v.gso_size,
                  csum_start=v.csum_start, csum_offset=v.csum_offset)
    return st, a, out[: r.out_len if (st == 0 and not r.passthrough) else 0], vafter, res


GSO_DESC = np.dtype([("in_offset", "<u8"), ("out_offset", "<u8"), ("in_len", "<u4"), ("out_cap", "<u4"),
                     ("vnet", VNET_HDR), ("reserved", "<u2", 3)])
assert GSO_DESC.itemsize == 40


def gso_split_desc(inbuf: np.ndarray, desc: np.ndarray, outbuf: np.ndarray, threads: int | None = None):
    """do_tun_gso_split for a batch of 40-byte descriptors, in place on inbuf
    (the reference zeroes prefix fields) and into outbuf; returns statuses."""
    a, o = _u8(inbuf), _u8(outbuf)
    d = np.ascontiguousarray(desc).view(GSO_DESC).reshape(-1)
    end_in = int((d["in_offset"] + d["in_len"]).max()) if d.size else 0
    end_out = int((d["out_offset"] + d["out_cap"]).max()) if d.size else 0
    if end_in > a.size or end_out > o.size:
        raise ValueError("gso_split_desc: descriptor past a buffer")
    st = np.zeros(d.size, dtype=np.int8)
    lib.orc_gso_split_desc(a.ctypes.data, d.ctypes.data, d.size, o.ctypes.data, st.ctypes.data,
                           threads or default_threads())
    return st


def time_l4_uniform(buf: np.ndarray, segment_size: int, csum_start: int, flags: int, threads: int,
                    reps: int) -> float:
    a = _u8(buf)
    n = (a.size + segment_size - 1) // segment_size
    out = np.empty(n, dtype=np.uint16)
    return float(lib.orc_time_l4_uniform(a.ctypes.data, a.size, segment_size, csum_start, flags,
                                         out.ctypes.data, threads, reps))


# ---------------------------------------------------------------------------
# data-message AEAD: oracle/aead_oracle.c
# ---------------------------------------------------------------------------
REJECT_AFTER_MESSAGES = (1 << 64) - 1 - (1 << 13)  # include/proto/proto.hpp:36


def _b(x) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8) if not isinstance(x, np.ndarray) else x,
                                dtype=np.uint8)


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    out = np.zeros(64, np.uint8)
    k, n = _b(key), _b(nonce)
    lib.orc_chacha20_block(k.ctypes.data, counter, n.ctypes.data, out.ctypes.data)
    return out.tobytes()


def poly1305(key: bytes, msg: bytes) -> bytes:
    out = np.zeros(16, np.uint8)
    k, m = _b(key), _b(msg)
    lib.orc_poly1305(k.ctypes.data, m.ctypes.data, m.size, out.ctypes.data)
    return out.tobytes()


def aead_encrypt(key: bytes, nonce: bytes, aad: bytes, pt: bytes):
    k, n, a, p = _b(key), _b(nonce), _b(aad), _b(pt)
    ct = np.zeros(max(p.size, 1), np.uint8)
    tag = np.zeros(16, np.uint8)
    lib.orc_aead_encrypt(k.ctypes.data, n.ctypes.data, a.ctypes.data, a.size, p.ctypes.data, p.size, ct.ctypes.data,
                         tag.ctypes.data)
    return ct[: p.size].tobytes(), tag.tobytes()


def aead_decrypt(key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
    k, n, a, c, t = _b(key), _b(nonce), _b(aad), _b(ct), _b(tag)
    pt = np.full(max(c.size, 1), 0xEE, np.uint8)
    rc = lib.orc_aead_decrypt(k.ctypes.data, n.ctypes.data, a.ctypes.data, a.size, c.ctypes.data, c.size,
                              t.ctypes.data, pt.ctypes.data)
    return rc, pt[: c.size].tobytes()


def wg_encrypt(key: bytes, receiver_index: int, counter: int, pt: bytes) -> bytes:
    k, p = _b(key), _b(pt)
    out = np.zeros(16 + (p.size + 15) // 16 * 16 + 16, np.uint8)
    n = lib.orc_wg_encrypt(k.ctypes.data, receiver_index, counter, p.ctypes.data, p.size, out.ctypes.data)
    return out[:n].tobytes()


def wg_decrypt(key: bytes, msg: bytes):
    k, m = _b(key), _b(msg)
    out = np.full(max(m.size - 32, 1), 0xEE, np.uint8)
    rc = lib.orc_wg_decrypt(k.ctypes.data, m.ctypes.data, m.size, out.ctypes.data)
    return rc, out[: max(m.size - 32, 0)].tobytes()


def wg_encrypt_batch(key: bytes, receiver_index: int, counter0: int, buf: np.ndarray, segment_size: int) -> np.ndarray:
    """Every segment of a PacketBatch into consecutive data messages at the
    stride expected_encrypt_size(segment_size) (worker/encap.cpp:136-141)."""
    k, a = _b(key), _u8(buf)
    n = (a.size + segment_size - 1) // segment_size
    stride = 16 + (segment_size + 15) // 16 * 16 + 16
    last = a.size - (n - 1) * segment_size if n else 0
    out = np.zeros(max((n - 1) * stride + 16 + (last + 15) // 16 * 16 + 16, 1) if n else 1, np.uint8)
    lib.orc_wg_encrypt_batch(k.ctypes.data, receiver_index, counter0, a.ctypes.data, a.size, segment_size,
                             out.ctypes.data)
    return out[: (n - 1) * stride + 16 + (last + 15) // 16 * 16 + 16] if n else out[:0]


def wg_decrypt_batch(key: bytes, buf: np.ndarray, segment_size: int):
    """Every message of a GRO batch (worker/decap_ref.cpp:78-86); plaintext i at
    i * (segment_size - 32); status 0 / -1 per message."""
    k, a = _b(key), _u8(buf)
    n = (a.size + segment_size - 1) // segment_size
    ostride = max(segment_size - 32, 0)
    out = np.full(max(n * ostride, 1), 0xEE, np.uint8)
    st = np.zeros(max(n, 1), np.int8)
    lib.orc_wg_decrypt_batch(k.ctypes.data, a.ctypes.data, a.size, segment_size, out.ctypes.data, st.ctypes.data)
    return out[: n * ostride], st[:n]


def wg_encrypt_batch_mt(key: bytes, receiver_index: int, counter0: int, buf: np.ndarray, segment_size: int,
                        out: np.ndarray, threads: int) -> None:
    """wg_encrypt_batch into a preallocated `out`, over host threads (the
    CPU baseline's timed call)."""
    k, a = _b(key), _u8(buf)
    lib.orc_wg_encrypt_batch_mt(k.ctypes.data, receiver_index, counter0, a.ctypes.data, a.size, segment_size,
                                out.ctypes.data, threads)


def wg_decrypt_batch_mt(key: bytes, buf: np.ndarray, segment_size: int, out: np.ndarray, status: np.ndarray,
                        threads: int) -> None:
    k, a = _b(key), _u8(buf)
    lib.orc_wg_decrypt_batch_mt(k.ctypes.data, a.ctypes.data, a.size, segment_size, out.ctypes.data,
                                status.ctypes.data, threads)


_OSS = None


def _oss():
    global _OSS
    if _OSS is None:
        path = HERE / "build" / "libaead_openssl.so"
        if not path.exists():
            build()
        _OSS = ctypes.CDLL(str(path))
        _OSS.oss_wg_encrypt_batch.restype = ctypes.c_int
        _OSS.oss_wg_encrypt_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        _OSS.oss_wg_decrypt_batch.restype = ctypes.c_int
        _OSS.oss_wg_decrypt_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return _OSS


def openssl_encrypt_batch(key: bytes, receiver_index: int, counter0: int, buf: np.ndarray, segment_size: int,
                          out: np.ndarray, threads: int) -> None:
    """The same batch over the system OpenSSL's EVP_chacha20_poly1305
    (oracle/openssl_aead.c): an optimised RFC 8439 of libsodium's class, the
    f4 CPU comparator."""
    _oss()
    k, a = _b(key), _u8(buf)
    rc = _OSS.oss_wg_encrypt_batch(k.ctypes.data, receiver_index, counter0, a.ctypes.data, a.size, segment_size,
                                   out.ctypes.data, threads)
    if rc != 0:
        raise RuntimeError("OpenSSL EVP_chacha20_poly1305 failed")


def openssl_decrypt_batch(key: bytes, buf: np.ndarray, segment_size: int, out: np.ndarray, status: np.ndarray,
                          threads: int) -> None:
    """Peer::decrypt per message of a GRO batch over OpenSSL's
    EVP_chacha20_poly1305 (the decap CPU comparator): plaintext i at
    i * (segment_size - 32) of `out`, status 0 / -1 per message."""
    _oss()
    k, a = _b(key), _u8(buf)
    n = (a.size + segment_size - 1) // segment_size
    assert out.size >= n * max(segment_size - 32, 0) and status.size >= n and status.dtype == np.int8
    rc = _OSS.oss_wg_decrypt_batch(k.ctypes.data, a.ctypes.data, a.size, segment_size, out.ctypes.data,
                                   status.ctypes.data, threads)
    if rc != 0:
        raise RuntimeError("OpenSSL EVP_chacha20_poly1305 failed")
