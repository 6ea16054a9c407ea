#!/usr/bin/env python3
"""Sustained-rate study: per-launch kernel times over many back-to-back
launches of the L4 kernel and of the read probe (same bytes), to separate
kernel behaviour from the memory system's sustained rate.
  python tools/sustain.py [--launches 400]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--workload", default="config2")
    args = ap.parse_args()
    import torch

    import bench
    import wireglider_amd as wga

    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, args.workload, 0, 1, dev)
    launch, payload, alg = wl.launch, wl.payload_bytes, wl.alg_bytes
    buf = torch.empty(payload // 16 * 16, dtype=torch.uint8, device=dev)
    buf.fill_(3)
    acc = torch.zeros(1, dtype=torch.int64, device=dev)

    def series(fn, k):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        return [round(e0.elapsed_time(e1) * 1e3, 1) for e0, e1 in ev]

    out = {}
    for name, fn, nbytes in (("l4", launch, alg), ("probe_2k", lambda: wga.probe_read(buf, acc, 2), buf.numel()),
                             ("probe_4k", lambda: wga.probe_read(buf, acc, 4), buf.numel()),
                             ("probe_8k", lambda: wga.probe_read(buf, acc, 8), buf.numel()),
                             ("l4_again", launch, alg)):
        s = series(fn, args.launches)
        bins = [round(sum(s[i:i + 20]) / len(s[i:i + 20]), 1) for i in range(0, len(s), 20)]
        out[name] = {"us_per_launch_binned20": bins, "first10": s[:10],
                     "GBps_first10": round(nbytes / (sum(s[:10]) / 10 * 1e-6) / 1e9, 1),
                     "GBps_last100": round(nbytes / (sum(s[-100:]) / 100 * 1e-6) / 1e9, 1)}
        torch.cuda.synchronize()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
