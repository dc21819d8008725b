"""Build libkdstep.so (gfx950) in-tree with hipcc.

Each .hip translation unit is compiled to an object in parallel (objects are
cached by source mtime + header mtimes), then linked into one shared library that
exports exactly the extern "C" symbols of include/kdstep.h.  No torch headers are
involved: the library is a plain C-ABI .so loaded with ctypes.

    python csrc/build.py          the product library (package dir)
    python csrc/build.py --ab     tools/ab/libkdstep_ab.so: the same sources with -DKD_AB_BUILD, i.e.
                                  also the negative-result / diagnostic kernels and the A/B switches
                                  (v9, v11, v12, stamp builds, attention variants, ab_knob env vars);
                                  tools and tools/ab_tests load it with KD_LIBRARY=<path>
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
AB_LIB = REPO / "tools" / "ab" / "libkdstep_ab.so"
AB_OBJ_DIR = HERE / "build_ab"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable", "-ffp-contract=fast",
          f"-I{REPO / 'include'}"]


def _sources():
    return sorted(HERE.glob("*.hip"))


def _deps_mtime(ab: bool = False):
    hdrs = list(HERE.glob("*.h")) + list((REPO / "include").glob("*.h")) + [Path(__file__)]
    if ab:
        hdrs += list(AB_LIB.parent.glob("*.inc"))
    return max(p.stat().st_mtime for p in hdrs)


def _compile(src: Path, ab: bool = False) -> Path:
    obj = (AB_OBJ_DIR if ab else OBJ_DIR) / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, _deps_mtime(ab)):
        return obj
    # the A/B-only kernel bodies live in tools/ab/*.inc, included inside the sources' KD_AB_BUILD blocks
    cmd = [HIPCC, *CFLAGS, *(["-DKD_AB_BUILD", f"-I{AB_LIB.parent}"] if ab else []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int | None = None, ab: bool = False) -> Path:
    lib = AB_LIB if ab else LIB
    (AB_OBJ_DIR if ab else OBJ_DIR).mkdir(exist_ok=True)
    lib.parent.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s_: _compile(s_, ab), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if lib.exists() and lib.stat().st_mtime > newest:
        if not ab:
            _try_c_host(verbose)
        return lib
    # the A/B library also links hipBLASLt (tools/ab/gemm_blas.inc); the product library links no BLAS
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(lib),
           *(["-L/opt/rocm/lib", "-lhipblaslt"] if ab else [])]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {lib}")
    if not ab:
        _try_c_host(verbose)
    return lib


def _try_c_host(verbose: bool) -> None:
    """The C-host example is not part of the library: build it when its source is shipped,
    and only warn when it does not compile."""
    if not C_HOST_SRC.exists():
        return
    try:
        build_c_host(verbose)
    except RuntimeError as e:   # pragma: no cover - an example build failure is not fatal
        print(f"warning: {e}", file=sys.stderr)


C_HOST_SRC = REPO / "tools" / "c_host_step.cpp"
C_HOST_BIN = OUT_DIR / "kd_c_host_step"


def build_c_host(verbose: bool = False) -> Path:
    """The C-ABI host example (tools/c_host_step.cpp: a full KD step with no Python), linked
    against libkdstep.so next to it (rpath $ORIGIN)."""
    if C_HOST_BIN.exists() and C_HOST_BIN.stat().st_mtime > max(C_HOST_SRC.stat().st_mtime, LIB.stat().st_mtime):
        return C_HOST_BIN
    cmd = [HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", f"-I{REPO / 'include'}", str(C_HOST_SRC),
           f"-L{OUT_DIR}", "-lkdstep", "-Wl,-rpath,$ORIGIN", "-o", str(C_HOST_BIN)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"c host build failed:\n{r.stderr}")
    if verbose:
        print(f"built {C_HOST_BIN}")
    return C_HOST_BIN


if __name__ == "__main__":
    build(verbose=True, ab="--ab" in sys.argv[1:])
    sys.exit(0)
