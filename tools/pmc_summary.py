#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced
streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE (KiB) is
taken as is.  Writes a JSON summary next to the CSVs and prints it.
usage: pmc_summary.py <outdir> [bench args...]
"""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path


def per_kernel(path_glob):
    """Kernel name -> list of per-dispatch counter values."""
    vals = {}
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                vals.setdefault(row.get("Kernel_Name", ""), []).append(float(row["Counter_Value"]))
    return vals


# the kernels one step of each workload launches (substrings of the kernel
# names); their per-dispatch medians add up to the step's HBM bytes
STEP_KERNELS = {
    "config1": ["l4csum_coop_kernel"],
    "config2": ["l4csum_kernel<"],
    "config3": ["gso_plan_kernel", "gso_split_kernel", "gso_finalize_kernel"],
    "config3udp": ["gso_plan_kernel", "gso_split_kernel", "gso_finalize_kernel"],
    "config4": ["l4csum_split_kernel"],
    "config4strong": ["l4csum_split_kernel"],
    "config4small": ["l4csum_split_kernel"],
    "config5": ["l4csum_split_kernel"],
    "verify": ["verify_kernel<"],
    "verify64d": ["verify_walk_kernel<true>"],  # all-small batches: the walking kernel, consecutive layout (the spread one runs only on the first calls)
    "verify64": ["verify_"],
    "verify1500u": ["verify_"],
    "gro": ["gro_finalize"],
    "aead": ["aead_kernel"],
    "encap": ["gso_plan_kernel", "gso_split_kernel", "gso_finalize_kernel", "encap_scan", "aead_kernel"],
}


def main():
    out = Path(sys.argv[1])
    args = sys.argv[2:]
    workload = "config2"
    if "--workload" in args:
        workload = args[args.index("--workload") + 1]
    res = {"workload": workload, "bench_args": args, "kernels": {}}
    f_all = per_kernel(str(out / "pmc_FETCH_SIZE" / "**" / "*counter_collection.csv"))
    w_all = per_kernel(str(out / "pmc_WRITE_SIZE" / "**" / "*counter_collection.csv"))
    subs = STEP_KERNELS.get(workload, ["l4csum_kernel<"])
    rd = wr = 0.0
    for name, f in sorted(f_all.items()):
        if not any(x in name for x in subs):
            continue
        fk = statistics.median(f)
        w = w_all.get(name, [])
        wk = statistics.median(w) if w else 0.0
        res["kernels"][name] = {
            "dispatches": len(f),
            "FETCH_SIZE_KiB_median": fk,
            "WRITE_SIZE_KiB_median": wk,
            "read_bytes_corrected": 2 * fk * 1024,
            "write_bytes": wk * 1024,
        }
        rd += 2 * fk * 1024
        wr += wk * 1024
    if res["kernels"]:
        res["read_bytes_per_launch"] = rd
        res["write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
    res["correction"] = "gfx950: read bytes = 2 x FETCH_SIZE KiB x 1024 (MI355X_MICROARCH.md §HBM); write = WRITE_SIZE KiB x 1024"
    if workload == "gro":
        res["calibration_note"] = ("gro_finalize stages its header chunks with 16 B/lane loads, consecutive lanes on "
                                   "consecutive chunks of a flow (contiguous for the bench's 64 B slots), plus 24 B "
                                   "descriptors: the x2 read correction is calibrated for coalesced 16 B/lane streams; "
                                   "raw FETCH_SIZE is kept above")
    (out / f"pmc_{workload}.json").write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
