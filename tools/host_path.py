#!/usr/bin/env python3
"""Host-memory path rate: the batch starts and ends in host
memory (tun / UDP socket buffers), so the end-to-end rate includes the H2D
copy of the packets and the D2H copy of the 2-byte results.

On BASELINE config 2 bytes (1,048,576 x 1500 B), one process:
  pipeline_pageable : wg_l4csum_uniform_host on a pageable numpy buffer
                      (the library's chunked two-stream pipeline; the HIP
                      runtime stages the pageable source)
  pipeline_pinned   : the same entry point on wg_host_alloc memory (DMA
                      straight from the caller's buffer)
  h2d_hip_pinned    : hipMemcpyAsync of the whole pinned buffer alone, through
                      libamdhip64 on a fresh stream (the copy the pipeline issues)
  h2d_hip_pageable  : the same from the pageable buffer
  h2d_hip_torch_pinned_buffer : hipMemcpyAsync from a torch pin_memory buffer
  h2d_torch_pinned  : torch's tensor.copy_(pinned, non_blocking=True) from that
                      buffer — round 1's "h2d_only", which came out slower than
                      the whole library path
The pipeline runs at chunk sizes 8 MiB .. 2 GiB (knob host_chunk_mb; 2 GiB =
one chunk, no overlap).  Every rate is bytes / wall time of 5 repetitions
after one warm-up; every library result is checked against the device batch
entry point's.
"""
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    import wireglider_amd as wga

    n, seg = 1 << 20, 1500
    nbytes = n * seg
    dev = torch.device("cuda:0")
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    wga.synth_fill(d, 0x5EED0002)
    desc = wga.synth_desc_stride(n, seg, seg, 0, 0x5EED0002, 0, device=dev)
    wga.synth_headers(d, desc, 0x5EED0002, 0)
    torch.cuda.synchronize()
    pageable = d.cpu().numpy()
    pinned = wga.PinnedBuffer(nbytes)
    pinned.array[:] = pageable
    dev_ref = wga.calc_l4_checksum_batch(d, seg, False, False, 20).cpu().numpy()

    def rate(fn, reps=5):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        return {"ms": round(dt * 1e3, 3), "GBps": round(nbytes / dt / 1e9, 2), "GiBps": round(nbytes / dt / 2**30, 2)}

    out = {"batch_bytes": nbytes}
    chunk0 = wga.tune_get("host_chunk_mb")
    for mb in (8, 32, 128, 512, 2048):
        wga.tune_set("host_chunk_mb", mb)
        for name, arr in (("pipeline_pageable", pageable), ("pipeline_pinned", pinned.array)):
            got = wga.calc_l4_checksum_host(arr, seg, False, False, 20)
            assert np.array_equal(got, dev_ref), name
            out[f"{name}_chunk{mb}MiB"] = rate(lambda: wga.calc_l4_checksum_host(arr, seg, False, False, 20))
    wga.tune_set("host_chunk_mb", chunk0)

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    st = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    h2d = 1  # hipMemcpyHostToDevice

    def hip_copy(src_ptr):
        def f():
            assert hip.hipMemcpyAsync(d.data_ptr(), src_ptr, nbytes, h2d, st) == 0
            assert hip.hipStreamSynchronize(st) == 0
        return f

    out["h2d_hip_pinned"] = rate(hip_copy(pinned.array.ctypes.data))
    out["h2d_hip_pageable"] = rate(hip_copy(pageable.ctypes.data))
    tp = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)  # torch's own pinned allocation (round 1)
    tp.copy_(torch.from_numpy(pageable))
    out["h2d_hip_torch_pinned_buffer"] = rate(hip_copy(tp.data_ptr()))

    def torch_copy():
        d.copy_(tp, non_blocking=True)
        torch.cuda.synchronize()

    out["h2d_torch_pinned"] = rate(torch_copy)
    pinned.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
