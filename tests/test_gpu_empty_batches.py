"""Empty batches and refused arguments on every batch entry point of the C ABI.

The reference's callers hand over whatever a tun read or a recvmmsg returned,
including nothing: an empty PacketBatch has nr_segments() == 0
(include/util/packets.hpp:11-47, include/worker/offload.hpp:26-28), and
do_tun_gso_split / evaluate_packet are simply not called for it.  Here an
empty call returns WG_OK, queues nothing that writes, and leaves every output
byte as it was.  The one output that does change is wg_encap_batch /
wg_encap_encrypt's `dev_total`, which becomes 0 (no messages: counter0 +
*dev_total is still the peer's next nonce, worker/encap.cpp:136-141).  A
refused call (null / misaligned pointers with n > 0) returns WG_ERR_INVALID
and writes nothing either.  Every check runs on a side stream filled with a
sentinel first."""
import ctypes

import numpy as np
import pytest

SENT = 0x5A
KEY = bytes(range(32))


def _wga():
    import wireglider_amd as wga

    return wga


@pytest.fixture
def bufs(gpu):
    import torch

    s = torch.cuda.Stream(gpu)
    b = {k: torch.full((4096,), SENT, dtype=torch.uint8, device=gpu) for k in
         ("base", "desc", "out", "out2", "out3", "res", "work", "total", "msgs", "off")}
    torch.cuda.synchronize()
    return s, b


def _unchanged(b, skip=()):
    import torch

    torch.cuda.synchronize()
    for k, t in b.items():
        if k not in skip:
            assert bool((t == SENT).all()), f"{k} was written"


def _p(t, off=0):
    return t.data_ptr() + off


@pytest.mark.gpu
def test_empty_device_batches_write_nothing(bufs):
    wga = _wga()
    L = wga.lib
    s, b = bufs
    st = ctypes.c_void_p(s.cuda_stream)
    calls = {
        "wg_l4csum_uniform": lambda: L.wg_l4csum_uniform(_p(b["base"]), 0, 1500, 20, 0, _p(b["out"]), st),
        "wg_l4csum_desc": lambda: L.wg_l4csum_desc(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), st),
        "wg_checksum_desc": lambda: L.wg_checksum_desc(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), st),
        "wg_verify_desc": lambda: L.wg_verify_desc(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), _p(b["out2"]), st),
        "wg_verify_uniform": lambda: L.wg_verify_uniform(_p(b["base"]), 0, 64, _p(b["out"]), _p(b["out2"]), st),
        "wg_gso_split": lambda: L.wg_gso_split(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), _p(b["res"]), st),
        "wg_gro_finalize": lambda: L.wg_gro_finalize(_p(b["base"]), _p(b["desc"]), 0, st),
        "wg_aead_encrypt_batch": lambda: L.wg_aead_encrypt_batch(_p(b["base"]), 0, 1500, KEY, 7, 0, _p(b["out"]),
                                                                 _p(b["out2"]), st),
        "wg_aead_decrypt_batch": lambda: L.wg_aead_decrypt_batch(_p(b["base"]), 0, 1532, KEY, _p(b["out"]),
                                                                 _p(b["out2"]), st),
        "wg_aead_decrypt_verify_batch": lambda: L.wg_aead_decrypt_verify_batch(
            _p(b["base"]), 0, 1532, KEY, _p(b["out"]), _p(b["out2"]), _p(b["out3"]), _p(b["res"]), st),
        "wg_synth_fill": lambda: L.wg_synth_fill(_p(b["base"]), 0, 1, 0, st),
        "wg_synth_headers": lambda: L.wg_synth_headers(_p(b["base"]), _p(b["desc"]), 0, 1, 0, st),
        "wg_synth_desc_stride": lambda: L.wg_synth_desc_stride(_p(b["desc"]), 0, 1500, 1500, 0, 1, 0, st),
        "wg_store_l4csum": lambda: L.wg_store_l4csum(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), st),
    }
    for name, call in calls.items():
        assert call() == 0, name
    _unchanged(b)


@pytest.mark.gpu
@pytest.mark.parametrize("entry", ["wg_encap_batch", "wg_encap_encrypt"])
def test_empty_encap_reports_zero_messages(bufs, entry):
    """n = 0: no message written, no result record, and *dev_total = 0 (it
    held a stale count before the call)."""
    import torch

    wga = _wga()
    s, b = bufs
    st = ctypes.c_void_p(s.cuda_stream)
    fn = getattr(wga.lib, entry)
    if entry == "wg_encap_batch":
        rc = fn(_p(b["base"]), _p(b["desc"]), 0, _p(b["out"]), _p(b["res"]), KEY, 7, 100, _p(b["off"]), 1536, 45,
                1460, _p(b["msgs"]), _p(b["out2"]), _p(b["work"]), _p(b["total"]), st)
    else:
        rc = fn(_p(b["base"]), _p(b["out"]), _p(b["desc"]), _p(b["res"]), 0, KEY, 7, 100, _p(b["off"]), 1536, 45,
                1460, _p(b["msgs"]), _p(b["out2"]), _p(b["work"]), _p(b["total"]), st)
    assert rc == 0
    _unchanged(b, skip=("total",))
    assert int(b["total"][:8].view(torch.int64).item()) == 0
    assert bool((b["total"][8:] == SENT).all())


@pytest.mark.gpu
def test_refused_arguments_write_nothing(bufs):
    """n > 0 with a null or misaligned pointer: WG_ERR_INVALID before any
    launch, so the other (valid) outputs keep their bytes."""
    wga = _wga()
    L = wga.lib
    s, b = bufs
    st = ctypes.c_void_p(s.cuda_stream)
    inval = {
        "wg_l4csum_uniform null out": lambda: L.wg_l4csum_uniform(_p(b["base"]), 3000, 1500, 20, 0, None, st),
        "wg_l4csum_uniform segment 0": lambda: L.wg_l4csum_uniform(_p(b["base"]), 3000, 0, 20, 0, _p(b["out"]), st),
        "wg_l4csum_desc misaligned": lambda: L.wg_l4csum_desc(_p(b["base"]), _p(b["desc"], 8), 4, _p(b["out"]), st),
        "wg_checksum_desc null base": lambda: L.wg_checksum_desc(None, _p(b["desc"]), 4, _p(b["out"]), st),
        "wg_verify_desc misaligned": lambda: L.wg_verify_desc(_p(b["base"]), _p(b["desc"], 4), 4, _p(b["out"]),
                                                              _p(b["out2"]), st),
        "wg_verify_desc null verdict": lambda: L.wg_verify_desc(_p(b["base"]), _p(b["desc"]), 4, None,
                                                                _p(b["out2"]), st),
        "wg_verify_uniform null verdict": lambda: L.wg_verify_uniform(_p(b["base"]), 640, 64, None, _p(b["out2"]),
                                                                      st),
        "wg_gso_split null res": lambda: L.wg_gso_split(_p(b["base"]), _p(b["desc"]), 2, _p(b["out"]), None, st),
        "wg_gso_split misaligned desc": lambda: L.wg_gso_split(_p(b["base"]), _p(b["desc"], 4), 2, _p(b["out"]),
                                                               _p(b["res"]), st),
        "wg_gro_finalize null desc": lambda: L.wg_gro_finalize(_p(b["base"]), None, 2, st),
        "wg_aead_encrypt_batch misaligned out": lambda: L.wg_aead_encrypt_batch(
            _p(b["base"]), 3000, 1500, KEY, 7, 0, _p(b["out"], 4), _p(b["out2"]), st),
        "wg_aead_encrypt_batch null key": lambda: L.wg_aead_encrypt_batch(
            _p(b["base"]), 3000, 1500, None, 7, 0, _p(b["out"]), _p(b["out2"]), st),
        "wg_aead_decrypt_batch null status": lambda: L.wg_aead_decrypt_batch(
            _p(b["base"]), 3064, 1532, KEY, _p(b["out"]), None, st),
        "wg_aead_decrypt_verify_batch null l4": lambda: L.wg_aead_decrypt_verify_batch(
            _p(b["base"]), 3064, 1532, KEY, _p(b["out"]), _p(b["out2"]), _p(b["out3"]), None, st),
        "wg_encap_batch null work": lambda: L.wg_encap_batch(
            _p(b["base"]), _p(b["desc"]), 2, _p(b["out"]), _p(b["res"]), KEY, 7, 100, _p(b["off"]), 1536, 45, 1460,
            _p(b["msgs"]), _p(b["out2"]), None, _p(b["total"]), st),
        "wg_encap_encrypt max_segments 0": lambda: L.wg_encap_encrypt(
            _p(b["base"]), _p(b["out"]), _p(b["desc"]), _p(b["res"]), 2, KEY, 7, 100, _p(b["off"]), 1536, 0, 1460,
            _p(b["msgs"]), _p(b["out2"]), _p(b["work"]), _p(b["total"]), st),
    }
    for name, call in inval.items():
        assert call() == -1, name
    _unchanged(b)


@pytest.mark.gpu
def test_empty_host_batches(gpu):
    """The host-memory entry points: an empty batch returns WG_OK without
    touching the outputs; wg_encap_host reports next_counter = counter0."""
    wga = _wga()
    L = wga.lib
    src = np.full(4096, SENT, np.uint8)
    outs = [np.full(4096, SENT, np.uint8) for _ in range(4)]
    p = [o.ctypes.data for o in outs]
    assert L.wg_l4csum_uniform_host(src.ctypes.data, 0, 1500, 20, 0, p[0]) == 0
    assert L.wg_decap_host(src.ctypes.data, 0, 1532, KEY, p[0], p[1], p[2], p[3]) == 0
    nxt = ctypes.c_uint64(0xDEAD)
    assert L.wg_encap_host(src.ctypes.data, p[0], 0, KEY, 7, 12345, 45, 1460, 1536, p[1], p[2], p[3],
                           ctypes.byref(nxt)) == 0
    assert nxt.value == 12345
    # refused: verdict without l4, msg_cap not a multiple of 16
    assert L.wg_decap_host(src.ctypes.data, 3064, 1532, KEY, p[0], p[1], p[2], None) == -1
    assert L.wg_encap_host(src.ctypes.data, p[0], 1, KEY, 7, 0, 45, 1460, 1530, p[1], p[2], p[3], None) == -1
    for o in outs:
        assert (o == SENT).all()
