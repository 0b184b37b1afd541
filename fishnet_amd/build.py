"""Builds libgpu_nnue.so in-tree for gfx950 (hipcc, no JIT, no torch extension).

Output: fishnet_amd/lib/libgpu_nnue.so (git-ignored; travels to the GPU box with
the gpurun snapshot).  Run: python -m fishnet_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libgpu_nnue.so")
SOURCES = ["gpu_nnue.hip", "kernels.hip", "stream.hip"]
HEADERS = ["chess.h", "host_board.h", "nnue.h", "kernels.h", "sha256.h", "device_util.h", "archive.h"]
ARCH = "gfx950"


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "gpu_nnue.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """defines/out: experiment variants (e.g. -DGN_EXPAND_WPE=5 into lib/libgpu_nnue_w5.so),
    selected at run time with GPU_NNUE_LIB; the default build has neither."""
    lib = out or LIB
    if not force and not defines and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    objs = []
    for src in SOURCES:
        obj = os.path.join(LIBDIR, src.replace(".hip", f".{os.getpid()}.o"))
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
               "-Wall", "-Wno-unused-function", *defines, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + f".tmp{os.getpid()}"
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    outs = [a[len("--out="):] for a in sys.argv[1:] if a.startswith("--out=")]
    print(build(force="--force" in sys.argv, verbose=True, defines=defs,
                out=os.path.join(LIBDIR, outs[0]) if outs else None))
