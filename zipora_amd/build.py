"""Builds libzipora_amd.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m zipora_amd.build            # incremental
    python -m zipora_amd.build --force
    python -m zipora_amd.build --diag     # tools-only build with the profiling
                                          # ablations (-DZR_DIAG): libzipora_amd_diag.so
"""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "_obj")
LIB = os.path.join(PKG, "libzipora_amd.so")
OBJ_DIAG = os.path.join(PKG, "_obj_diag")
LIB_DIAG = os.path.join(PKG, "libzipora_amd_diag.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ZR_OFFLOAD_ARCH", "gfx950")

SOURCES = ["zr_api.cpp", "zr_rans.hip", "zr_fse.hip", "zr_huff.hip", "zr_pipe.cpp", "zr_compressor.hip",
           "zr_comm.cpp"]
HEADERS = ["zr_internal.h", os.path.join("..", "..", "include", "zipora_amd.h")]
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable", "-munsafe-fp-atomics"]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src, diag=False):
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ_DIAG if diag else OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS]
    if not _newer(o, deps):
        return o
    cmd = [HIPCC] + CFLAGS + (["-DZR_DIAG"] if diag else []) + ["-x", "hip", "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return o


def build(force=False, verbose=False, diag=False):
    obj_dir, lib = (OBJ_DIAG, LIB_DIAG) if diag else (OBJ, LIB)
    os.makedirs(obj_dir, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    if force:
        for s in srcs:
            p = os.path.join(obj_dir, s + ".o")
            if os.path.exists(p):
                os.remove(p)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, diag), srcs))
    if _newer(lib, objs) or force:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", lib] + objs + ["-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    if verbose:
        print(lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv)
