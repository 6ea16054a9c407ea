#!/usr/bin/env python3
"""Where config 5's distance to its read probe goes: one 16 M x 1500 B
buffer, one process, interleaved rounds of
  uniform   calc_l4_checksum_batch (PacketBatch, v4/UDP, csum_start 20)
  desc_v4   calc_l4_checksum_desc, every descriptor v4/UDP at csum_start 20
  desc_mix  the config 5 descriptors (v4/v6 x TCP/UDP mixed)
  probe     the kernel-shaped read probe over the same buffer (1500-B runs)
Prints one JSON object: median ms and GB/s of algorithmic bytes.
usage: desc_overhead.py [packets]
"""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import wireglider_amd as wga

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    seg = 1500
    dev = torch.device("cuda:0")
    buf = torch.empty(n * seg, dtype=torch.uint8, device=dev)
    wga.synth_fill(buf, 5)
    d_mix = wga.synth_desc_stride(n, seg, seg, 1, 5, 0, device=dev)
    d_v4 = wga.synth_desc_stride(n, seg, seg, 0, 5, 0, device=dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    acc = torch.zeros(1, dtype=torch.int64, device=dev)
    step = (4 << 30) // (16 * seg) * 16 * seg
    views = [buf[o: o + min(step, buf.numel() - o) // 16 * 16] for o in range(0, buf.numel(), step)]

    def probe():
        for v in views:
            wga.probe_read(v, acc, 1, run_bytes=seg)

    fns = {
        "uniform": (lambda: wga.calc_l4_checksum_batch(buf, seg, False, False, 20, out=out), n * (seg + 2)),
        "desc_v4": (lambda: wga.calc_l4_checksum_desc(buf, d_v4, out=out), n * (seg + 18)),
        "desc_mix": (lambda: wga.calc_l4_checksum_desc(buf, d_mix, out=out), n * (seg + 18)),
        "probe": (probe, n * seg),
    }
    t = {k: [] for k in fns}
    for _ in range(4):
        for k, (f, _) in fns.items():
            f()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for e0, e1 in ev:
                e0.record()
                f()
                e1.record()
            torch.cuda.synchronize()
            t[k] += [a.elapsed_time(b) for a, b in ev]
    res = {k: {"ms_med": round(statistics.median(v), 4),
               "GBps": round(fns[k][1] / (statistics.median(v) * 1e-3) / 1e9, 1)} for k, v in t.items()}
    print(json.dumps({"packets": n, "segment": seg, "variants": res}), flush=True)


if __name__ == "__main__":
    main()
