"""Build libmmt_hip.so (all HIP kernels + the C ABI of include/mmt_api.h) for gfx950.

Plain hipcc, no torch headers: each ``*.hip`` is compiled to an object (in parallel, incremental on
mtimes of the sources and headers) and linked into ``libmmt_hip.so`` next to this package, so the
library travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

CSRC = Path(__file__).resolve().parent
PKG = CSRC.parent
ROOT = PKG.parent
OBJ = CSRC / "_obj"
LIB = PKG / "libmmt_hip.so"
ARCH = "gfx950"

COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
                "-munsafe-fp-atomics"]
# Files whose bit-exact contract forbids FMA contraction (ToMe canonical arithmetic).
NO_CONTRACT = {"tome.hip"}
# Per-file extra flags. attention.hip: no NaN semantics (every NaN there would be a bug) and the
# IEEE mode bit off, so fmaxf on MFMA outputs is one v_max (no canonicalising v_max x, x first).
EXTRA = {"attention.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee"]}


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (Path(c).exists() or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _headers():
    return list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))


def _compile(src: Path) -> Path:
    obj = OBJ / (src.stem + ".o")
    deps = [src] + _headers()
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    flags = list(COMMON_FLAGS)
    flags.append("-ffp-contract=off" if src.name in NO_CONTRACT else "-ffp-contract=fast")
    flags += EXTRA.get(src.name, [])
    cmd = [_hipcc(), *flags, "-I", str(ROOT / "include"), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    if LIB.exists() and LIB.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return LIB
    cmd = [_hipcc(), "-shared", f"--offload-arch={ARCH}", "-o", str(LIB), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
