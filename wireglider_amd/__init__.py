"""wireglider_amd — MI355X-native Internet-checksum engine (Python plumbing).

The engine itself is C++/HIP (libwireglider_amd.so, C ABI in
include/wireglider_amd.h).  This module binds that ABI with ctypes and takes
torch tensors for device memory and streams; torch is plumbing only.

Mirrors the reference's interface for the path (dinhngtu/wireglider
@ 2024-11-01):
  calc_l4_checksum_batch  <- checksum.cpp:8-36 over a PacketBatch
                             (include/worker/offload.hpp:19-29)
  calc_l4_checksum_desc   <- the same over a descriptor batch
  checksum_desc           <- include/netio/checksum.hpp:146-149
  gso_split               <- worker/offload.cpp:46-216 (batched)

There is no CPU fallback: importing without the built library raises, and
every compute call requires a HIP device.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "lib" / "libwireglider_amd.so"
# A/B tooling only (tools/ab_builds.sh): load another build of the same library.
if os.environ.get("WG_LIB"):
    LIB_PATH = Path(os.environ["WG_LIB"]).resolve()

WG_OK = 0
WG_PKT_V6 = 0x01
WG_PKT_TCP = 0x02
WG_PROBE_DEFAULT_POLICY = 0x100  # wg_probe_copy: default cache policy instead of non-temporal
ABI_VERSION = 2

# Every symbol declared in include/wireglider_amd.h.
EXPORTED_SYMBOLS = (
    "wg_l4csum_uniform",
    "wg_l4csum_desc",
    "wg_checksum_desc",
    "wg_verify_desc",
    "wg_verify_uniform",
    "wg_gso_split",
    "wg_gro_finalize",
    "wg_aead_encrypt_batch",
    "wg_aead_decrypt_batch",
    "wg_aead_decrypt_verify_batch",
    "wg_encap_encrypt",
    "wg_encap_batch",
    "wg_l4csum_uniform_host",
    "wg_decap_host",
    "wg_encap_host",
    "wg_host_release",
    "wg_percall_stats",
    "wg_host_alloc",
    "wg_host_free",
    "wg_synth_fill",
    "wg_synth_headers",
    "wg_synth_desc_stride",
    "wg_store_l4csum",
    "wg_abi_version",
    "wg_strerror",
    "wg_device_count",
    "wg_tune_set",
    "wg_tune_get",
    "wg_probe_read",
    "wg_probe_copy",
)

# struct layouts (include/wireglider_amd.h)
PKT_DESC_BYTES = 16
GSO_DESC_BYTES = 40
GSO_RESULT_BYTES = 24
GRO_DESC_BYTES = 24


def _np_dtypes():
    import numpy as np

    pkt = np.dtype([("offset", "<u8"), ("len", "<u4"), ("csum_start", "<u2"), ("flags", "u1"),
                    ("reserved", "u1")])
    vnet = np.dtype([("flags", "u1"), ("gso_type", "u1"), ("hdr_len", "<u2"), ("gso_size", "<u2"),
                     ("csum_start", "<u2"), ("csum_offset", "<u2")])
    gso = np.dtype([("in_offset", "<u8"), ("out_offset", "<u8"), ("in_len", "<u4"), ("out_cap", "<u4"),
                    ("vnet", vnet), ("reserved", "<u2", 3)])
    res = np.dtype([("out_len", "<u8"), ("segment_size", "<u4"), ("hdr_len", "<u2"), ("isv6", "u1"),
                    ("ecn", "u1"), ("status", "i1"), ("passthrough", "u1"), ("pad", "u1", 6)])
    gro = np.dtype([("hdr_offset", "<u8"), ("payload_bytes", "<u8"), ("hdr_len", "<u2"), ("csum_start", "<u2"),
                    ("csum_offset", "<u2"), ("flags", "u1"), ("status", "i1")])
    assert pkt.itemsize == PKT_DESC_BYTES and gso.itemsize == GSO_DESC_BYTES and res.itemsize == GSO_RESULT_BYTES
    assert gro.itemsize == GRO_DESC_BYTES
    return pkt, gso, res, gro


PKT_DESC_DTYPE, GSO_DESC_DTYPE, GSO_RESULT_DTYPE, GRO_DESC_DTYPE = _np_dtypes()


class WireGliderError(RuntimeError):
    pass


def _load() -> ctypes.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(wireglider_amd has no CPU fallback)"
        )
    lib = ctypes.CDLL(str(LIB_PATH))
    u8p = ctypes.c_void_p
    vp = ctypes.c_void_p
    u64 = ctypes.c_uint64
    u32 = ctypes.c_uint32
    u16 = ctypes.c_uint16
    i32 = ctypes.c_int
    sig = {
        "wg_l4csum_uniform": (i32, [u8p, u64, u32, u16, u32, vp, vp]),
        "wg_l4csum_desc": (i32, [u8p, vp, u64, vp, vp]),
        "wg_checksum_desc": (i32, [u8p, vp, u64, vp, vp]),
        "wg_verify_desc": (i32, [u8p, vp, u64, vp, vp, vp]),
        "wg_verify_uniform": (i32, [u8p, u64, u32, vp, vp, vp]),
        "wg_gso_split": (i32, [u8p, vp, u64, u8p, vp, vp]),

        "wg_gro_finalize": (i32, [u8p, vp, u64, vp]),
        "wg_aead_encrypt_batch": (i32, [u8p, u64, u32, ctypes.c_char_p, u32, u64, u8p, vp, vp]),
        "wg_aead_decrypt_batch": (i32, [u8p, u64, u32, ctypes.c_char_p, u8p, vp, vp]),
        "wg_aead_decrypt_verify_batch": (i32, [u8p, u64, u32, ctypes.c_char_p, u8p, vp, vp, vp, vp]),
        "wg_encap_encrypt": (i32, [u8p, u8p, vp, vp, u64, ctypes.c_char_p, u32, u64, vp, u32, u32, u32, u8p, vp, vp,
                                   vp, vp]),
        "wg_encap_batch": (i32, [u8p, vp, u64, u8p, vp, ctypes.c_char_p, u32, u64, vp, u32, u32, u32, u8p, vp, vp, vp,
                                 vp]),
        "wg_l4csum_uniform_host": (i32, [u8p, u64, u32, u16, u32, vp]),
        "wg_decap_host": (i32, [u8p, u64, u32, ctypes.c_char_p, vp, vp, vp, vp]),
        "wg_encap_host": (i32, [u8p, vp, u64, ctypes.c_char_p, u32, u64, u32, u32, u32, vp, vp, vp,
                                ctypes.POINTER(u64)]),
        "wg_host_release": (i32, []),
        "wg_percall_stats": (i32, [ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "wg_host_alloc": (i32, [ctypes.POINTER(ctypes.c_void_p), u64]),
        "wg_host_free": (i32, [vp]),
        "wg_synth_fill": (i32, [u8p, u64, u64, u64, vp]),
        "wg_synth_headers": (i32, [u8p, vp, u64, u64, u64, vp]),
        "wg_synth_desc_stride": (i32, [vp, u64, u64, u32, i32, u64, u64, vp]),
        "wg_store_l4csum": (i32, [u8p, vp, u64, vp, vp]),
        "wg_abi_version": (i32, []),
        "wg_strerror": (ctypes.c_char_p, [i32]),
        "wg_device_count": (i32, []),
        "wg_tune_set": (i32, [ctypes.c_char_p, u64]),
        "wg_tune_get": (i32, [ctypes.c_char_p, ctypes.POINTER(u64)]),
        "wg_probe_read": (i32, [u8p, u64, vp, u32, u32, vp]),
        "wg_probe_copy": (i32, [u8p, u8p, u64, u32, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.wg_abi_version() != ABI_VERSION:
        raise ImportError(f"ABI mismatch: library {lib.wg_abi_version()} != {ABI_VERSION}")
    return lib


lib = _load()


def _check(rc: int, what: str) -> None:
    if rc != WG_OK:
        raise WireGliderError(f"{what}: {lib.wg_strerror(rc).decode()} ({rc})")


# ---------------------------------------------------------------------------
# torch plumbing
# ---------------------------------------------------------------------------


def _torch():
    import torch

    return torch


def _stream_ptr(stream, tensor=None) -> int | None:
    """The launch stream: `stream`, else the current stream of the device
    that holds `tensor` (not of whichever device happens to be current)."""
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream(tensor.device if tensor is not None else None)
    return stream.cuda_stream


def _on(t):
    """Launch on the device that holds `t` (HIP launches go to the current
    device)."""
    return _torch().cuda.device(t.device)


def _check_out(out, n: int, dtype, like, name: str) -> None:
    """A caller-supplied output must hold n elements of `dtype` on the same
    device: an undersized tensor would be an out-of-bounds device write."""
    _require_cuda(out, name)
    if out.dtype != dtype or out.device != like.device:
        raise WireGliderError(f"{name}: expected {dtype} on {like.device}, got {out.dtype} on {out.device}")
    if out.numel() < n:
        raise WireGliderError(f"{name}: {out.numel()} elements, the batch needs {n}")


def _require_cuda(t, name: str):
    if not t.is_cuda:
        raise WireGliderError(f"{name} must be a device tensor (wireglider_amd has no CPU path)")
    if not t.is_contiguous():
        raise WireGliderError(f"{name} must be contiguous")


def nr_segments(total_len: int, segment_size: int) -> int:
    """PacketBatch::nr_segments (include/worker/offload.hpp:26-28)."""
    return (total_len + segment_size - 1) // segment_size


def calc_l4_checksum_batch(batch, segment_size: int, isv6: bool, istcp: bool, csum_start: int,
                           out=None, stream=None):
    """calc_l4_checksum (checksum.cpp:8-36) for every segment of a PacketBatch.

    batch: 1-D uint8 device tensor = PacketBatch.data; segment i is
    batch[i*S : min((i+1)*S, len)].  Returns a uint16 device tensor.
    """
    torch = _torch()
    _require_cuda(batch, "batch")
    n = nr_segments(batch.numel(), segment_size)
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=batch.device)
    _check_out(out, n, torch.uint16, batch, "out")
    flags = (WG_PKT_V6 if isv6 else 0) | (WG_PKT_TCP if istcp else 0)
    with _on(batch):
        rc = lib.wg_l4csum_uniform(batch.data_ptr(), batch.numel(), segment_size, csum_start, flags,
                                   out.data_ptr(), _stream_ptr(stream, batch))
    _check(rc, "wg_l4csum_uniform")
    return out


def calc_l4_checksum_desc(base, desc, out=None, stream=None):
    """calc_l4_checksum per descriptor.  desc: (n, 16) uint8 or (n, 2) int64
    device tensor in wg_pkt_desc layout."""
    torch = _torch()
    _require_cuda(base, "base")
    _require_cuda(desc, "desc")
    n = desc.numel() * desc.element_size() // PKT_DESC_BYTES
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=base.device)
    _check_out(out, n, torch.uint16, base, "out")
    with _on(base):
        rc = lib.wg_l4csum_desc(base.data_ptr(), desc.data_ptr(), n, out.data_ptr(), _stream_ptr(stream, base))
    _check(rc, "wg_l4csum_desc")
    return out


def checksum_desc(base, desc, out=None, stream=None):
    """checksum(span, 0) (include/netio/checksum.hpp:146-149) per descriptor."""
    torch = _torch()
    _require_cuda(base, "base")
    _require_cuda(desc, "desc")
    n = desc.numel() * desc.element_size() // PKT_DESC_BYTES
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=base.device)
    _check_out(out, n, torch.uint16, base, "out")
    with _on(base):
        rc = lib.wg_checksum_desc(base.data_ptr(), desc.data_ptr(), n, out.data_ptr(), _stream_ptr(stream, base))
    _check(rc, "wg_checksum_desc")
    return out


VERDICT_IP_OK, VERDICT_L4_OK, VERDICT_TCP, VERDICT_UDP, VERDICT_V6 = 0x01, 0x02, 0x04, 0x08, 0x10


def verify_desc(base, desc, with_l4: bool = True, stream=None, verdict=None, l4=None):
    """Decap verify gates (evaluate_packet's checksum decisions,
    include/worker/evaluator.hpp:112-149) per descriptor.  Returns
    (verdict uint8 tensor, L4 result uint16 tensor or None); preallocated
    outputs may be passed in."""
    torch = _torch()
    _require_cuda(base, "base")
    _require_cuda(desc, "desc")
    n = desc.numel() * desc.element_size() // PKT_DESC_BYTES
    if verdict is None:
        verdict = torch.empty(n, dtype=torch.uint8, device=base.device)
    if l4 is None and with_l4:
        l4 = torch.empty(n, dtype=torch.uint16, device=base.device)
    _check_out(verdict, n, torch.uint8, base, "verdict")
    if l4 is not None:
        _check_out(l4, n, torch.uint16, base, "l4")
    with _on(base):
        rc = lib.wg_verify_desc(base.data_ptr(), desc.data_ptr(), n, verdict.data_ptr(),
                                l4.data_ptr() if l4 is not None else None, _stream_ptr(stream, base))
    _check(rc, "wg_verify_desc")
    return verdict, l4


def verify_uniform(batch, segment_size: int, with_l4: bool = True, stream=None, verdict=None, l4=None):
    """Decap verify gates over a uniform PacketBatch (segment i =
    batch[i*S : min((i+1)*S, len)]), e.g. the plaintexts of one UDP GRO batch.
    Returns (verdict uint8 tensor, L4 result uint16 tensor or None)."""
    torch = _torch()
    _require_cuda(batch, "batch")
    n = nr_segments(batch.numel(), segment_size)
    if verdict is None:
        verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=batch.device)[:n]
    if l4 is None and with_l4:
        l4 = torch.empty(max(n, 1), dtype=torch.uint16, device=batch.device)[:n]
    _check_out(verdict, n, torch.uint8, batch, "verdict")
    if l4 is not None:
        _check_out(l4, n, torch.uint16, batch, "l4")
    with _on(batch):
        rc = lib.wg_verify_uniform(batch.data_ptr(), batch.numel(), segment_size, verdict.data_ptr(),
                                   l4.data_ptr() if l4 is not None else None, _stream_ptr(stream, batch))
    _check(rc, "wg_verify_uniform")
    return verdict, l4


def gso_split(inbuf, gso_desc, outbuf, results=None, stream=None):
    """Batched do_tun_gso_split (worker/offload.cpp:46-216).  gso_desc:
    device tensor of n x 40 B wg_gso_desc; results: n x 24 B wg_gso_result."""
    torch = _torch()
    for t, nm in ((inbuf, "inbuf"), (gso_desc, "gso_desc"), (outbuf, "outbuf")):
        _require_cuda(t, nm)
    n = gso_desc.numel() * gso_desc.element_size() // GSO_DESC_BYTES
    if results is None:
        results = torch.zeros(n * GSO_RESULT_BYTES, dtype=torch.uint8, device=inbuf.device)
    _check_out(results, n * GSO_RESULT_BYTES, torch.uint8, inbuf, "results")
    if gso_desc.device != inbuf.device or outbuf.device != inbuf.device:
        raise WireGliderError("gso_split: inbuf, gso_desc and outbuf must be on one device")
    with _on(inbuf):
        rc = lib.wg_gso_split(inbuf.data_ptr(), gso_desc.data_ptr(), n, outbuf.data_ptr(),
                              results.data_ptr(), _stream_ptr(stream, inbuf))
    _check(rc, "wg_gso_split")
    return results


def gro_finalize(hdrs, gro_desc, stream=None):
    """Batched GRO finalize (include/worker/flowkey_ref.hpp:82-117) in place on
    header buffers; gro_desc: device tensor of n x 24 B wg_gro_desc (status
    written back)."""
    for t, nm in ((hdrs, "hdrs"), (gro_desc, "gro_desc")):
        _require_cuda(t, nm)
    n = gro_desc.numel() * gro_desc.element_size() // GRO_DESC_BYTES
    if gro_desc.device != hdrs.device:
        raise WireGliderError("gro_finalize: hdrs and gro_desc must be on one device")
    with _on(hdrs):
        rc = lib.wg_gro_finalize(hdrs.data_ptr(), gro_desc.data_ptr(), n, _stream_ptr(stream, hdrs))
    _check(rc, "wg_gro_finalize")


def aead_message_stride(segment_size: int) -> int:
    """Peer::expected_encrypt_size(segment_size) (include/proto/proto.hpp:266-269)."""
    return 16 + (segment_size + 15) // 16 * 16 + 16


def aead_encrypt_batch(batch, segment_size: int, key: bytes, receiver_index: int, counter0: int, out=None,
                       status=None, stream=None):
    """Peer::encrypt (proto/proto.cpp:544-583) for every segment of a
    PacketBatch (worker/encap.cpp:136-141): message i at i * stride of `out`
    (uint8 device tensor), counter counter0 + i.  Returns (out, status)."""
    torch = _torch()
    _require_cuda(batch, "batch")
    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    n = nr_segments(batch.numel(), segment_size)
    last = batch.numel() - (n - 1) * segment_size if n else 0
    need = (n - 1) * aead_message_stride(segment_size) + aead_message_stride(last) if n else 0
    if out is None:
        out = torch.empty(max(need, 1), dtype=torch.uint8, device=batch.device)
    _check_out(out, need, torch.uint8, batch, "out")
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.int8, device=batch.device)
    _check_out(status, n, torch.int8, batch, "status")
    with _on(batch):
        rc = lib.wg_aead_encrypt_batch(batch.data_ptr(), batch.numel(), segment_size, bytes(key), receiver_index,
                                       counter0 & (2**64 - 1), out.data_ptr(), status.data_ptr(),
                                       _stream_ptr(stream, batch))
    _check(rc, "wg_aead_encrypt_batch")
    return out, status


def aead_decrypt_batch(msgs, segment_size: int, key: bytes, out=None, status=None, stream=None):
    """Peer::decrypt (proto/proto.cpp:496-523) for every message of a batch
    of equal-size data messages (worker/decap_ref.cpp:78-86): plaintext i at
    i * (segment_size - 32) of `out`.  Returns (out, status)."""
    torch = _torch()
    _require_cuda(msgs, "msgs")
    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    n = nr_segments(msgs.numel(), segment_size)
    need = n * max(segment_size - 32, 0)
    if out is None:
        out = torch.empty(max(need, 1), dtype=torch.uint8, device=msgs.device)
    _check_out(out, need, torch.uint8, msgs, "out")
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.int8, device=msgs.device)
    _check_out(status, n, torch.int8, msgs, "status")
    with _on(msgs):
        rc = lib.wg_aead_decrypt_batch(msgs.data_ptr(), msgs.numel(), segment_size, bytes(key), out.data_ptr(),
                                       status.data_ptr(), _stream_ptr(stream, msgs))
    _check(rc, "wg_aead_decrypt_batch")
    return out, status


def aead_decrypt_verify_batch(msgs, segment_size: int, key: bytes, out=None, status=None, verdict=None, l4=None,
                              stream=None):
    """aead_decrypt_batch and, in the same pass, the decap verify gates
    (wg_verify_desc, evaluate_packet: include/worker/evaluator.hpp:112-149)
    over every plaintext at its libsodium (padded) length, as
    worker/decap_ref.cpp:81-86 evaluates it.  Returns (out, status, verdict,
    l4)."""
    torch = _torch()
    _require_cuda(msgs, "msgs")
    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    n = nr_segments(msgs.numel(), segment_size)
    need = n * max(segment_size - 32, 0)
    if out is None:
        out = torch.empty(max(need, 1), dtype=torch.uint8, device=msgs.device)
    _check_out(out, need, torch.uint8, msgs, "out")
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.int8, device=msgs.device)
    _check_out(status, n, torch.int8, msgs, "status")
    if verdict is None:
        verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=msgs.device)
    _check_out(verdict, n, torch.uint8, msgs, "verdict")
    if l4 is None:
        l4 = torch.empty(max(n, 1), dtype=torch.uint16, device=msgs.device)
    _check_out(l4, n, torch.uint16, msgs, "l4")
    with _on(msgs):
        rc = lib.wg_aead_decrypt_verify_batch(msgs.data_ptr(), msgs.numel(), segment_size, bytes(key),
                                              out.data_ptr(), status.data_ptr(), verdict.data_ptr(), l4.data_ptr(),
                                              _stream_ptr(stream, msgs))
    _check(rc, "wg_aead_decrypt_verify_batch")
    return out, status, verdict, l4


ENCAP_RESULT_BYTES = 16


def _encap_dtype():
    import numpy as np

    d = np.dtype([("counter0", "<u8"), ("nmsg", "<u4"), ("msg_bytes", "<u4")])
    assert d.itemsize == ENCAP_RESULT_BYTES
    return d


ENCAP_RESULT_DTYPE = _encap_dtype()


def _encap_outputs(inbuf, gso_desc, gso_results, key, msg_offset, results, work, total):
    """Shared argument checks / default outputs of encap_encrypt and encap_batch."""
    torch = _torch()
    _require_cuda(inbuf, "inbuf")
    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    n = gso_desc.numel() * gso_desc.element_size() // GSO_DESC_BYTES
    _check_out(gso_results, n * GSO_RESULT_BYTES, torch.uint8, inbuf, "gso_results")
    _check_out(msg_offset, n, torch.int64, inbuf, "msg_offset")
    if results is None:
        results = torch.zeros(max(n, 1) * ENCAP_RESULT_BYTES, dtype=torch.uint8, device=inbuf.device)
    _check_out(results, n * ENCAP_RESULT_BYTES, torch.uint8, inbuf, "results")
    if work is None:
        work = torch.empty(n + 1024, dtype=torch.int32, device=inbuf.device)
    _check_out(work, n + 1024, torch.int32, inbuf, "work")
    if total is None:
        total = torch.zeros(1, dtype=torch.int64, device=inbuf.device)
    _check_out(total, 1, torch.int64, inbuf, "total")
    return n, results, work, total


def _encap_buffers(inbuf, out, out_name, gso_desc, msgs, msg_offset, msg_cap: int, n: int) -> None:
    """The byte buffers of an encap call: uint8 on inbuf's device.  The caller
    owns the message extent (msg_offset[i] + msg_cap <= msgs.numel(), every
    msg_offset[i] a multiple of 16, as include/wireglider_amd.h documents); it
    is checked here only with WG_DEBUG_CHECKS=1 in the environment (the check
    copies msg_offset to the host and waits for it)."""
    import numpy as np

    torch = _torch()
    for t, nm in ((out, out_name), (msgs, "msgs"), (gso_desc, "gso_desc")):
        _require_cuda(t, nm)
        if t.device != inbuf.device:
            raise WireGliderError(f"{nm}: expected a tensor on {inbuf.device}, got {t.device}")
    for t, nm in ((out, out_name), (msgs, "msgs")):
        if t.dtype != torch.uint8:
            raise WireGliderError(f"{nm}: expected torch.uint8, got {t.dtype}")
    if n and msgs.numel() < msg_cap:
        raise WireGliderError(f"msgs: {msgs.numel()} bytes, smaller than one super-buffer's msg_cap {msg_cap}")
    if n and os.environ.get("WG_DEBUG_CHECKS") == "1":
        offs = msg_offset[:n].to("cpu").numpy().astype(np.uint64)
        if (offs % 16).any():
            raise WireGliderError("msg_offset: every entry must be a multiple of 16")
        if int(offs.max()) + msg_cap > msgs.numel():
            raise WireGliderError(f"msgs: {msgs.numel()} bytes, msg_offset + msg_cap reaches {int(offs.max()) + msg_cap}")


def encap_encrypt(inbuf, seg_out, gso_desc, gso_results, key: bytes, receiver_index: int, counter0: int, msg_offset,
                  msg_cap: int, max_segments: int, max_segment_size: int, msgs, results=None, work=None, total=None,
                  stream=None):
    """Encap worker step (worker/encap.cpp:136-141) after gso_split: every
    segment of every super-buffer's PacketBatch encrypted for one peer, with
    consecutive counters from counter0 in super-buffer / segment order,
    messages of super-buffer i at msg_offset[i] (uint64 device tensor).
    Returns (results uint8 tensor of wg_encap_result, total uint64 tensor)."""
    n, results, work, total = _encap_outputs(inbuf, gso_desc, gso_results, key, msg_offset, results, work, total)
    _encap_buffers(inbuf, seg_out, "seg_out", gso_desc, msgs, msg_offset, msg_cap, n)
    with _on(inbuf):
        rc = lib.wg_encap_encrypt(inbuf.data_ptr(), seg_out.data_ptr(), gso_desc.data_ptr(), gso_results.data_ptr(), n,
                                  bytes(key), receiver_index, counter0 & (2**64 - 1), msg_offset.data_ptr(), msg_cap,
                                  max_segments, max_segment_size, msgs.data_ptr(), results.data_ptr(),
                                  work.data_ptr(), total.data_ptr(), _stream_ptr(stream, inbuf))
    _check(rc, "wg_encap_encrypt")
    return results, total


def encap_batch(inbuf, gso_desc, out, gso_results, key: bytes, receiver_index: int, counter0: int, msg_offset,
                msg_cap: int, max_segments: int, max_segment_size: int, msgs, results=None, work=None, total=None,
                stream=None):
    """The whole encap step (worker/encap.cpp:107-168: do_tun_gso_split, then
    Peer::encrypt per segment) in one call: gso_split writing only the
    segments' headers into `out`, then encap_encrypt reading every segment's
    payload from `inbuf`.  Same results / messages / total as gso_split +
    encap_encrypt; `out` holds the segment headers only."""
    n, results, work, total = _encap_outputs(inbuf, gso_desc, gso_results, key, msg_offset, results, work, total)
    _encap_buffers(inbuf, out, "out", gso_desc, msgs, msg_offset, msg_cap, n)
    with _on(inbuf):
        rc = lib.wg_encap_batch(inbuf.data_ptr(), gso_desc.data_ptr(), n, out.data_ptr(), gso_results.data_ptr(),
                                bytes(key), receiver_index, counter0 & (2**64 - 1), msg_offset.data_ptr(), msg_cap,
                                max_segments, max_segment_size, msgs.data_ptr(), results.data_ptr(), work.data_ptr(),
                                total.data_ptr(), _stream_ptr(stream, inbuf))
    _check(rc, "wg_encap_batch")
    return results, total


def calc_l4_checksum_host(buf: bytes | bytearray | memoryview, segment_size: int, isv6: bool,
                          istcp: bool, csum_start: int):
    """Host-memory path: host buffer in, host uint16 array out (H2D, kernel, D2H)."""
    import numpy as np

    mv = np.frombuffer(buf, dtype=np.uint8)
    n = nr_segments(mv.size, segment_size)
    out = np.empty(n, dtype=np.uint16)
    flags = (WG_PKT_V6 if isv6 else 0) | (WG_PKT_TCP if istcp else 0)
    rc = lib.wg_l4csum_uniform_host(mv.ctypes.data, mv.size, segment_size, csum_start, flags,
                                    out.ctypes.data)
    _check(rc, "wg_l4csum_uniform_host")
    return out


def _host_u8(a, name):
    import numpy as np

    if not isinstance(a, np.ndarray) or a.dtype != np.uint8 or not a.flags.c_contiguous:
        raise WireGliderError(f"{name} must be a contiguous numpy uint8 array (host memory)")
    return a


def decap_host(msgs, segment_size: int, key: bytes, verify: bool = True, plain=None):
    """The decap worker's step on a UDP GRO batch in host memory
    (worker/decap_ref.cpp:53-89: Peer::decrypt, then evaluate_packet): msgs
    (numpy uint8, e.g. a PinnedBuffer's array) holds equal-size messages at
    stride segment_size.  Returns (plaintext uint8 array, status int8, verdict
    uint8 or None, l4 uint16 or None), as aead_decrypt_verify_batch would."""
    import numpy as np

    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    m = _host_u8(msgs, "msgs")
    n = nr_segments(m.size, segment_size)
    need = n * max(segment_size - 32, 0)
    if plain is None:
        plain = np.empty(max(need, 1), np.uint8)
    _host_u8(plain, "plain")
    if plain.size < need:
        raise WireGliderError(f"plain: {plain.size} bytes, the batch needs {need}")
    status = np.empty(max(n, 1), np.int8)
    verdict = np.empty(max(n, 1), np.uint8) if verify else None
    l4 = np.empty(max(n, 1), np.uint16) if verify else None
    rc = lib.wg_decap_host(m.ctypes.data, m.size, segment_size, bytes(key), plain.ctypes.data, status.ctypes.data,
                           verdict.ctypes.data if verify else None, l4.ctypes.data if verify else None)
    _check(rc, "wg_decap_host")
    return plain[:need], status[:n], (verdict[:n] if verify else None), (l4[:n] if verify else None)


def encap_host(inbuf, gso_desc, key: bytes, receiver_index: int, counter0: int, max_segments: int,
               max_segment_size: int, msg_cap: int, msgs=None):
    """The encap worker's step on tun reads in host memory (worker/encap.cpp:
    22-170): inbuf (numpy uint8) holds the super-buffers gso_desc (numpy
    GSO_DESC_DTYPE array) describes, in input order; super-buffer i's
    messages at msgs[i * msg_cap:].  Returns (msgs, results ENCAP_RESULT_DTYPE,
    gso results GSO_RESULT_DTYPE, next counter)."""
    import numpy as np

    if len(key) != 32:
        raise WireGliderError("key must be 32 bytes")
    a = _host_u8(inbuf, "inbuf")
    d = np.ascontiguousarray(gso_desc)
    if d.dtype != GSO_DESC_DTYPE:
        raise WireGliderError("gso_desc must be a GSO_DESC_DTYPE array")
    n = d.size
    if n and int((d["in_offset"] + d["in_len"]).max()) > a.size:
        raise WireGliderError("gso_desc reaches past inbuf")
    if msgs is None:
        msgs = np.empty(max(n * msg_cap, 1), np.uint8)
    _host_u8(msgs, "msgs")
    if msgs.size < n * msg_cap:
        raise WireGliderError(f"msgs: {msgs.size} bytes, the batch needs {n * msg_cap}")
    res = np.zeros(max(n, 1), ENCAP_RESULT_DTYPE)
    gres = np.zeros(max(n, 1), GSO_RESULT_DTYPE)
    nxt = ctypes.c_uint64(0)
    rc = lib.wg_encap_host(a.ctypes.data, d.ctypes.data, n, bytes(key), receiver_index, counter0 & (2**64 - 1),
                           max_segments, max_segment_size, msg_cap, msgs.ctypes.data, res.ctypes.data,
                           gres.ctypes.data, ctypes.byref(nxt))
    _check(rc, "wg_encap_host")
    return msgs, res[:n], gres[:n], int(nxt.value)


def host_release() -> None:
    """Free this thread's host-path workspace (rebuilt on next use)."""
    _check(lib.wg_host_release(), "wg_host_release")


class PinnedBuffer:
    """Pinned host memory from wg_host_alloc (the engine's packet I/O
    buffers), exposed as a numpy uint8 array; freed by close() / GC."""

    def __init__(self, nbytes: int):
        import numpy as np

        self._p = ctypes.c_void_p()
        _check(lib.wg_host_alloc(ctypes.byref(self._p), nbytes), "wg_host_alloc")
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self._p.value))

    def close(self) -> None:
        if self._p is not None and self._p.value:
            self.array = None
            _check(lib.wg_host_free(self._p), "wg_host_free")
        self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# synthetic batches (bench / tests)
# ---------------------------------------------------------------------------


def synth_fill(buf, seed: int, counter_base: int = 0, stream=None) -> None:
    _require_cuda(buf, "buf")
    with _on(buf):
        _check(lib.wg_synth_fill(buf.data_ptr(), buf.numel() * buf.element_size(), seed, counter_base,
                                 _stream_ptr(stream, buf)), "wg_synth_fill")


def synth_headers(base, desc, seed: int, index_base: int = 0, stream=None) -> None:
    n = desc.numel() * desc.element_size() // PKT_DESC_BYTES
    with _on(base):
        _check(lib.wg_synth_headers(base.data_ptr(), desc.data_ptr(), n, seed, index_base,
                                    _stream_ptr(stream, base)), "wg_synth_headers")


def synth_desc_stride(n: int, stride: int, length: int, mode: int, seed: int, index_base: int = 0,
                      device=None, stream=None):
    torch = _torch()
    desc = torch.empty((n, 2), dtype=torch.int64, device=device or "cuda")
    with _on(desc):
        _check(lib.wg_synth_desc_stride(desc.data_ptr(), n, stride, length, mode, seed, index_base,
                                        _stream_ptr(stream, desc)), "wg_synth_desc_stride")
    return desc


def store_l4csum(base, desc, csum, stream=None) -> None:
    n = desc.numel() * desc.element_size() // PKT_DESC_BYTES
    with _on(base):
        _check(lib.wg_store_l4csum(base.data_ptr(), desc.data_ptr(), n, csum.data_ptr(),
                                   _stream_ptr(stream, base)), "wg_store_l4csum")


def tune_set(key: str, value: int) -> None:
    """Launch-geometry knob (results never depend on it)."""
    _check(lib.wg_tune_set(key.encode(), int(value)), f"wg_tune_set({key})")


def tune_get(key: str) -> int:
    v = ctypes.c_uint64(0)
    _check(lib.wg_tune_get(key.encode(), ctypes.byref(v)), f"wg_tune_get({key})")
    return int(v.value)


def probe_read(buf, out, kib_per_wave: int = 4, stream=None, run_bytes: int = 0) -> None:
    """Launch the read-roofline probe over a device buffer (run_bytes > 0:
    the L4 kernel's issue structure over run_bytes-byte segments)."""
    with _on(buf):
        _check(lib.wg_probe_read(buf.data_ptr(), buf.numel() * buf.element_size(), out.data_ptr(), kib_per_wave,
                                 run_bytes, _stream_ptr(stream, buf)), "wg_probe_read")


def probe_copy(src, dst, kib_per_wave: int = 2, stream=None, default_policy: bool = False) -> None:
    """Launch the copy-roofline probe (dst = src) over device buffers:
    non-temporal loads and stores, or the default cache policy."""
    n = min(src.numel() * src.element_size(), dst.numel() * dst.element_size())
    with _on(src):
        _check(lib.wg_probe_copy(src.data_ptr(), dst.data_ptr(), n,
                                 kib_per_wave | (WG_PROBE_DEFAULT_POLICY if default_policy else 0),
                                 _stream_ptr(stream, src)), "wg_probe_copy")


def device_count() -> int:
    return int(lib.wg_device_count())
