"""Build the native library `libirx.so` in-tree with hipcc for gfx950 (no CMake, no JIT cache).

`python -m image_restoration_and_enhancement_amd.build` or `__graft_entry__.build()`.
Objects go to `<pkg>/build/`, the shared library to `<pkg>/libirx.so` (git-ignored, but it
travels to the GPU box with the repository snapshot).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG / "build"
LIB = PKG / "libirx.so"

ARCH = os.environ.get("IRX_OFFLOAD_ARCH", "gfx950")
BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
              "-Wno-unused-variable", "-Wno-unused-but-set-variable", f"-I{INCLUDE}"]
# -ffp-contract=off where a kernel must match a numpy / fp32 restatement operation for operation (no FMA
# fusion); attention: fmaxf without NaN-quieting canonicalisations
PER_FILE = {"elementwise.hip": ["-ffp-contract=off"],
            "attention.hip": ["-fno-honor-nans"],
            "filters.hip": ["-ffp-contract=off"],
            "degrade.hip": ["-ffp-contract=off"]}


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libirx.so)")


def sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _headers():
    return list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))


def _stale(obj: Path, src: Path, hdr_mtime: float) -> bool:
    return not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_mtime)


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(exist_ok=True)
    hdr_mtime = max((h.stat().st_mtime for h in _headers()), default=0.0)
    srcs = sources()
    todo = [s for s in srcs if force or _stale(BUILD / (s.name + ".o"), s, hdr_mtime)]

    def compile_one(src: Path):
        obj = BUILD / (src.name + ".o")
        cmd = [hipcc, *BASE_FLAGS, *PER_FILE.get(src.name, []), "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr[-6000:]}")
        if verbose:
            print(f"  built {src.name}", file=sys.stderr)
        return obj

    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(compile_one, todo))
    objs = [BUILD / (s.name + ".o") for s in srcs]
    if todo or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    t = build(force="--force" in sys.argv, verbose=True)
    print(t)
