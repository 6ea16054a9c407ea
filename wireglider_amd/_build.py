"""In-tree build of libwireglider_amd.so (gfx950) and the test oracle.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container and on the GPU box alike.  Objects and the shared library land in
wireglider_amd/lib/ (git-ignored, but shipped to the GPU box by gpurun).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = LIBDIR / "obj"
LIBNAME = "libwireglider_amd.so"
ARCH = os.environ.get("WG_OFFLOAD_ARCH", "gfx950")

SOURCES = ["l4csum.hip", "gso.hip", "gro.hip", "aead.hip", "synth.hip", "capi.hip", "hostpath.hip", "checksum.cpp"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build wireglider_amd)")


def _common_flags() -> list[str]:
    return [
        "-O3",
        "-std=c++20",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-Wall",
        "-Wno-unused-function",
        f"-I{ROOT / 'include'}",
        f"-I{CSRC}",
    ]


# Per-file code generation flags.  aead.hip (VALU-issue bound, waves stalled
# on dependent instructions): LLVM's max-ilp machine scheduler, -1.5 % on the
# encrypt kernel, -0.6 % on the encap step (profiles/r04_aead_carry_ilp_ab.txt);
# the HBM-bound kernels keep the default scheduler.
FILE_FLAGS = {"aead.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def _needs(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def build_lib(verbose: bool = False, jobs: int = 8) -> Path:
    hipcc = _hipcc()
    OBJDIR.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.hpp")) + list((ROOT / "include").rglob("*.h*"))
    objs = []
    cmds = []
    for src in SOURCES:
        s = CSRC / src
        if not s.exists():
            continue
        o = OBJDIR / (s.stem + ".o")
        objs.append(o)
        if _needs(o, [s] + headers):
            lang = [] if s.suffix == ".hip" else ["-x", "hip"]
            cmds.append([hipcc, *_common_flags(), *FILE_FLAGS.get(src, []), *lang, "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(cmds) or 1))) as ex:
        for err in ex.map(run, cmds):
            if verbose and err:
                print(err, file=sys.stderr)

    lib = LIBDIR / LIBNAME
    if _needs(lib, objs):
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(lib), *map(str, objs), "-lpthread"]
        run(cmd)
    return lib


HARNESSES = ["mt_batch"]  # tests/cpp/<name>.cpp -> tests/cpp/bin/<name> (test harnesses, not product)


def build_harnesses(verbose: bool = False) -> list[Path]:
    """The GPU test harnesses that drive the C ABI from several host threads
    (tests/test_mt_batch.py), built here rather than inside a GPU test."""
    hipcc = _hipcc()
    lib = LIBDIR / LIBNAME
    out = []
    for name in HARNESSES:
        src = ROOT / "tests" / "cpp" / f"{name}.cpp"
        exe = ROOT / "tests" / "cpp" / "bin" / name
        exe.parent.mkdir(parents=True, exist_ok=True)
        if _needs(exe, [src, lib, ROOT / "include" / "wireglider_amd.h"]):
            cmd = [hipcc, "-O2", "-std=c++20", f"--offload-arch={ARCH}", "-x", "hip", f"-I{ROOT / 'include'}", str(src),
                   f"-L{LIBDIR}", "-lwireglider_amd", f"-Wl,-rpath,{LIBDIR}", "-lpthread", "-o", str(exe)]
            if verbose:
                print(" ".join(cmd), flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"harness build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        out.append(exe)
    return out


def build_oracle(verbose: bool = False) -> None:
    """Build the CPU oracle (test infrastructure) and, when the reference is
    mounted, the reference-test golden driver into oracle/_ref/."""
    odir = ROOT / "oracle"
    r = subprocess.run(["make", "-C", str(odir)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"oracle build failed\n{r.stdout}\n{r.stderr}")
    if Path("/root/reference/tests/checksum_tests.hpp").exists():
        r = subprocess.run(["make", "-C", str(odir), "ref"], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"oracle/_ref build failed\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("oracle built", flush=True)


def main() -> None:
    verbose = "-v" in sys.argv
    build_oracle(verbose)
    print(build_lib(verbose))
    build_harnesses(verbose)


if __name__ == "__main__":
    main()
