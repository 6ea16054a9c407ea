#!/usr/bin/env python3
"""profiles/valu_<workload>.json from a tools/counters.sh summary.json: the
timed kernel's SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES per launch (per-
dispatch medians), its full symbol (bench.py prices the line's VALU issue
roofline only when that symbol is the kernel it times) and the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time, when both are given).
usage: valu_profile.py <summary.json> <workload> [kernel_ms]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    src, wl = Path(sys.argv[1]), sys.argv[2]
    kern_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
    s = json.loads(src.read_text())
    (name, c), = s["kernels"].items()
    out = {"kernel": name, "workload": wl,
           "valu_winst_per_launch": c["SQ_INSTS_VALU"], "salu_winst_per_launch": c.get("SQ_INSTS_SALU"),
           "valu_int64_winst_per_launch": c.get("SQ_INSTS_VALU_INT64"), "waves": c["SQ_WAVES"],
           "wave_cycles_quad": c.get("SQ_WAVE_CYCLES"), "wait_inst_any_quad": c.get("SQ_WAIT_INST_ANY"),
           "wait_any_quad": c.get("SQ_WAIT_ANY"), "grbm_gui_active": c.get("GRBM_GUI_ACTIVE"),
           "source": f"rocprofv3 --pmc, tools/counters.sh ({src.parent.name}), per-dispatch medians"}
    if kern_ms and c.get("GRBM_GUI_ACTIVE"):
        out["effective_clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (kern_ms * 1e-3) / 1e9, 3)
        out["kernel_ms_for_clock"] = kern_ms
    dst = ROOT / "profiles" / f"valu_{wl}.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(dst, json.dumps(out))


if __name__ == "__main__":
    main()
