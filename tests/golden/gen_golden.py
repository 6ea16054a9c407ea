"""Regenerate the reference golden vectors in tests/golden/ref/.

Runs oracle/_ref/ref_golden — a driver compiled (by oracle/Makefile) around
the reference's OWN test oracle, /root/reference/tests/checksum_tests.hpp
(checksum_ref1 :11-34, create_packet :36-42, create_packet_carry :44-48),
compiled where it lies.  Outputs are data only (inputs and expected 16-bit
results of tests/test-checksum.cpp:11-25), committed so the GPU box, which
has no /root/reference, can check against them.

    python tests/golden/gen_golden.py
"""
import hashlib
import json
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
OUT = HERE / "ref"


def main() -> None:
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
    OUT.mkdir(exist_ok=True)
    subprocess.run([str(ROOT / "oracle" / "_ref" / "ref_golden"), str(OUT)], check=True)
    manifest = {}
    for f in sorted(OUT.iterdir()):
        if f.suffix in (".bin", ".u16"):
            manifest[f.name] = hashlib.sha256(f.read_bytes()).hexdigest()
    r = np.fromfile(OUT / "ref1_random_1_1500.u16", dtype="<u2")
    c = np.fromfile(OUT / "ref1_carry_1_63.u16", dtype="<u2")
    manifest["anchors"] = {
        "random": {str(n): f"0x{int(r[n - 1]):04x}" for n in (1, 2, 3, 20, 64, 100, 1460, 1500)},
        "carry": {str(n): f"0x{int(c[n - 1]):04x}" for n in (1, 2, 16, 63)},
        "random_65536": f"0x{int(np.fromfile(OUT / 'ref1_random_65536.u16', dtype='<u2')[0]):04x}",
        "create_packet_prefix": (OUT / "create_packet_65536.bin").read_bytes()[:8].hex(),
    }
    manifest["generator"] = "oracle/_ref/ref_golden (reference tests/checksum_tests.hpp, compiled in place)"
    (OUT / "manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")
    print(json.dumps(manifest["anchors"], indent=1))


if __name__ == "__main__":
    main()
