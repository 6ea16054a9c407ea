#!/usr/bin/env python3
"""The first wg_verify_desc call on a fresh stream: for
1 M x 64 B and 1 M x 1500 B batches (mixed v4/v6 x TCP/UDP, valid checksums),
the device time of the FIRST call on each of several new streams (the
default kernel choice has no sample there) and of the calls after it, each
call bracketed by its own event pair; results checked against the first.
Prints one JSON line."""
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
    out = {}
    for size in (64, 1500):
        n, seed = 1 << 20, 0x5EED00F1
        buf = torch.empty(n * size, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, seed)
        desc = wga.synth_desc_stride(n, size, size, 1, seed, 0, device=dev)
        wga.synth_headers(buf, desc, seed, 0)
        wga.store_l4csum(buf, desc, wga.calc_l4_checksum_desc(buf, desc))
        verdict = torch.empty(n, dtype=torch.uint8, device=dev)
        l4 = torch.empty(n, dtype=torch.uint16, device=dev)
        bench.settle(torch, lambda: wga.verify_desc(buf, desc, verdict=verdict, l4=l4), 0.2)  # clocks, default stream
        ref = (verdict.clone(), l4.clone())
        first, later, exact = [], [], True
        for _ in range(8):
            s = torch.cuda.Stream(dev)
            times = []
            with torch.cuda.stream(s):
                for _ in range(6):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    wga.verify_desc(buf, desc, verdict=verdict, l4=l4)
                    e1.record(s)
                    s.synchronize()
                    times.append(e0.elapsed_time(e1))
                    exact = exact and bool(torch.equal(verdict, ref[0]) and torch.equal(l4, ref[1]))
            first.append(times[0])
            later += times[2:]
        alg = n * (size + 16 + 1 + 2)
        out[f"{size}B"] = {"packets": n, "first_call_ms_median": round(statistics.median(first), 5),
                           "first_call_ms": [round(x, 5) for x in first],
                           "later_calls_ms_median": round(statistics.median(later), 5),
                           "first_call_roofline_frac": round(alg / (statistics.median(first) * 1e-3) / 8e12, 4),
                           "later_roofline_frac": round(alg / (statistics.median(later) * 1e-3) / 8e12, 4),
                           "bit_exact_across_calls": exact,
                           "note": "one event pair per call (isolated launches), fresh torch stream per trial"}
        del buf, desc, verdict, l4
        torch.cuda.empty_cache()
    print(json.dumps({"verify_first_call": out}), flush=True)


if __name__ == "__main__":
    main()
