#!/usr/bin/env python3
"""Block-per-descriptor (l4_coop) vs split-role kernel on small descriptor
batches of one packet size each: where the crossover lies.

usage: coop_probe.py   (one GPU; prints one JSON object)
For each (n, packet bytes): median kernel ms of checksum_desc under the
split kernel (l4_coop = 0) and the coop kernel at 4 / 8 / 16 waves, interleaved.
"""
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import numpy as np
    import torch

    import wireglider_amd as wga

    dev = torch.device("cuda:0")
    variants = [("split", 0, 4), ("coop4", 1 << 20, 4), ("coop8", 1 << 20, 8), ("coop16", 1 << 20, 16)]
    out = {}
    for n, size in ((1024, 65536), (4096, 65536), (16384, 65536), (65536, 65536), (16384, 9000), (16384, 1500),
                    (65536, 1500), (16384, 64), (65536, 64), (262144, 1500)):
        buf = torch.empty(n * size, dtype=torch.uint8, device=dev)
        wga.synth_fill(buf, 7, counter_base=0)
        pd = np.zeros(n, dtype=wga.PKT_DESC_DTYPE)
        pd["offset"] = np.arange(n, dtype=np.uint64) * size
        pd["len"] = size
        desc = torch.from_numpy(pd.view(np.uint8).copy()).to(dev)
        res = torch.empty(n, dtype=torch.uint16, device=dev)
        t = {v[0]: [] for v in variants}
        ref = None
        for _ in range(3):
            for name, coop, w in variants:
                wga.tune_set("l4_coop", coop)
                wga.tune_set("l4_coop_waves", w)
                wga.checksum_desc(buf, desc, out=res)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
                for e0, e1 in ev:
                    e0.record()
                    wga.checksum_desc(buf, desc, out=res)
                    e1.record()
                torch.cuda.synchronize()
                t[name] += [a.elapsed_time(b) for a, b in ev]
                r = res.cpu()
                assert ref is None or torch.equal(r, ref), (n, size, name)
                ref = r
        out[f"{n}x{size}"] = {k: round(statistics.median(v), 4) for k, v in t.items()}
        del buf
    wga.tune_set("l4_coop", 0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
