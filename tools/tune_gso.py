#!/usr/bin/env python3
"""Interleaved A/B of GSO split launch variants (waves per block x segments
per wave step x blocks per super-buffer) on BASELINE config 3, one process,
one device.  (profiles/r01_tune_gso*.json were taken with the first kernel
version, whose third knob was the grid-y split.)"""
import itertools
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    import wireglider_amd as wga

    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, "config3", 0, 1, dev)
    launch, payload, alg = wl.launch, wl.payload_bytes, wl.alg_bytes
    torch.cuda.synchronize()
    variants = list(itertools.product([4, 8], [0, 1, 2], [1, 2, 3]))
    res = {v: [] for v in variants}
    bench.settle(torch, launch, 0.3)
    for _ in range(3):
        for v in variants:
            wga.tune_set("gso_waves", v[0])
            wga.tune_set("gso_spw", v[1])
            wga.tune_set("gso_groups", v[2])
            launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for e0, e1 in ev:
                e0.record()
                launch()
                e1.record()
            torch.cuda.synchronize()
            res[v] += [e0.elapsed_time(e1) for e0, e1 in ev]
    rows = [{"waves": v[0], "spw": v[1], "groups": v[2], "ms_med": round(statistics.median(t), 3),
             "GBps_med": round(alg / (statistics.median(t) * 1e-3) / 1e9, 1)} for v, t in res.items()]
    rows.sort(key=lambda r: r["ms_med"])
    out = {"workload": "config3", "alg_bytes": alg, "variants": rows}
    # A/B variants and a torch device-to-device copy of the same bytes
    best = rows[0]
    wga.tune_set("gso_waves", 4)
    wga.tune_set("gso_spw", best["spw"])
    wga.tune_set("gso_groups", best["groups"])
    abl = {}
    for a in (0, 1, 32):
        wga.tune_set("gso_ablate", a)
        launch()
        ts = []
        for _ in range(3):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for e0, e1 in ev:
                e0.record()
                launch()
                e1.record()
            torch.cuda.synchronize()
            ts += [e0.elapsed_time(e1) for e0, e1 in ev]
        abl[a] = round(statistics.median(ts), 3)
    wga.tune_set("gso_ablate", 0)
    out["ablation_ms"] = {"0 real": abl[0], "1 nt stores (correct variant)": abl[1],
                          "32 launch-order blocks (correct variant)": abl[32]}
    src = torch.empty(17_179_869_184 // 16 * 16 // 2, dtype=torch.int16, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    cb = src.numel() * 2
    out["torch_copy"] = {"bytes_each_way": cb, "ms_med": round(statistics.median(ts), 3),
                         "GBps_rw": round(2 * cb / (statistics.median(ts) * 1e-3) / 1e9, 1)}
    for kib in (1, 2, 4):
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            wga.probe_copy(src, dst, kib)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[f"probe_copy_{kib}k"] = {"ms_med": round(statistics.median(ts), 3),
                                     "GBps_rw": round(2 * cb / (statistics.median(ts) * 1e-3) / 1e9, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
