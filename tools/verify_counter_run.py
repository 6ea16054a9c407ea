"""Driver for tools/kernel_counters.sh: a few launches of one bench.py
workload (argv[1]), nothing else on the GPU."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import wireglider_amd as wga  # noqa: E402

dev = torch.device("cuda:0")
wl = bench.build_workload(wga, torch, sys.argv[1], 0, 1, dev)
for _ in range(5):
    wl.launch()
torch.cuda.synchronize()
