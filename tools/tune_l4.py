#!/usr/bin/env python3
"""Interleaved A/B of L4 checksum launch variants and the read-roofline probe,
in ONE process on one device (guide §5.4 rule 24).  Prints a JSON summary.

  python tools/tune_l4.py [--workload config2|config5|config4] [--rounds 3]
"""
import argparse
import itertools
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ppw", default="1,2,4,8")
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--blocks", default="1024,2048,4096,16384")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--descv", default="0")
    args = ap.parse_args()
    import torch

    import bench
    import wireglider_amd as wga

    dev = torch.device("cuda:0")
    wl = bench.build_workload(wga, torch, args.workload, 0, 1, dev)
    launch, payload, alg = wl.launch, wl.payload_bytes, wl.alg_bytes
    torch.cuda.synchronize()

    def timeit(fn, iters):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) for e0, e1 in ev]

    variants = list(itertools.product([int(x) for x in args.ppw.split(",")], [int(x) for x in args.nt.split(",")],
                                      [int(x) for x in args.blocks.split(",")], [int(x) for x in args.descv.split(",")]))
    res = {v: [] for v in variants}
    ref_out = None
    for r in range(args.rounds):
        for v in variants:
            ppw, nt, blocks, dv = v
            wga.tune_set("l4_descv", dv)
            wga.tune_set("l4_ppw", ppw)
            wga.tune_set("l4_nt", nt)
            wga.tune_set("l4_blocks", blocks)
            launch()
            res[v] += timeit(launch, args.iters)
    rows = []
    for v, ts in res.items():
        med = statistics.median(ts)
        rows.append({"ppw": v[0], "nt": v[1], "blocks": v[2], "descv": v[3], "ms_med": round(med, 4), "ms_min": round(min(ts), 4),
                     "GBps_med": round(alg / (med * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda x: x["ms_med"])
    out = {"workload": args.workload, "alg_bytes": alg, "variants": rows}

    if args.probe:
        buf = torch.empty(max(payload, 4 << 30) // 16 * 16, dtype=torch.uint8, device=dev)
        buf.fill_(1)
        acc = torch.zeros(1, dtype=torch.int64, device=dev)
        pr = []
        for kib in (1, 2, 4, 8):
            ts = []
            for _ in range(args.rounds):
                ts += timeit(lambda: wga.probe_read(buf, acc, kib), args.iters)
            med = statistics.median(ts)
            pr.append({"kib_per_wave": kib, "bytes": buf.numel(), "ms_med": round(med, 4),
                       "GBps_med": round(buf.numel() / (med * 1e-3) / 1e9, 1)})
        pr.sort(key=lambda x: -x["GBps_med"])
        out["probe_read"] = pr
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
