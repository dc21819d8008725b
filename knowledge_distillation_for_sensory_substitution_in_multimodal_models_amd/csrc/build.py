"""Build libkdstep.so (gfx950) in-tree with hipcc.

Each .hip translation unit is compiled to an object in parallel (objects are
cached by source mtime + header mtimes), then linked into one shared library that
exports exactly the extern "C" symbols of include/kdstep.h.  No torch headers are
involved: the library is a plain C-ABI .so loaded with ctypes.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
OUT_DIR = HERE.parent  # the package directory: the .so travels with the snapshot
LIB = OUT_DIR / "libkdstep.so"
OBJ_DIR = HERE / "build"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable", "-ffp-contract=fast",
          f"-I{REPO / 'include'}"]


def _sources():
    return sorted(HERE.glob("*.hip"))


def _deps_mtime():
    hdrs = list(HERE.glob("*.h")) + list((REPO / "include").glob("*.h")) + [Path(__file__)]
    return max(p.stat().st_mtime for p in hdrs)


def _compile(src: Path) -> Path:
    obj = OBJ_DIR / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, _deps_mtime()):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    OBJ_DIR.mkdir(exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if LIB.exists() and LIB.stat().st_mtime > newest:
        return LIB
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(LIB)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
