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


def per_dispatch(path_glob, kernel_sub):
    vals = []
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    out = Path(sys.argv[1])
    args = sys.argv[2:]
    workload = "config2"
    if "--workload" in args:
        workload = args[args.index("--workload") + 1]
    res = {"workload": workload, "bench_args": args}
    for kern in ("l4csum_kernel", "l4csum_split_kernel", "l4csum_coop_kernel", "gso_split_kernel", "verify_kernel", "gro_finalize",
                 "aead_kernel"):
        f = per_dispatch(str(out / "pmc_FETCH_SIZE" / "**" / "*counter_collection.csv"), kern)
        w = per_dispatch(str(out / "pmc_WRITE_SIZE" / "**" / "*counter_collection.csv"), kern)
        if not f:
            continue
        fk = statistics.median(f)
        wk = statistics.median(w) if w else 0.0
        res[kern] = {
            "dispatches": len(f),
            "FETCH_SIZE_KiB_median": fk,
            "WRITE_SIZE_KiB_median": wk,
            "read_bytes_corrected": 2 * fk * 1024,
            "write_bytes": wk * 1024,
            "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
        }
    main_k = {"config3": "gso_split_kernel", "config3udp": "gso_split_kernel", "verify": "verify_kernel",
              "gro": "gro_finalize", "config1": "l4csum_coop_kernel", "config4": "l4csum_split_kernel",
              "config5": "l4csum_split_kernel", "aead": "aead_kernel"}.get(workload, "l4csum_kernel")
    if main_k in res:
        res["hbm_bytes_per_launch"] = res[main_k]["hbm_bytes_per_launch"]
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
