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
# test-only variant: the plan reports an entry overflow for block 1 on its first launch in a process
# (stream.hip GN_FAULT_PLAN_BLOCK; tests/test_gpu_parity.py::test_plan_overflow_fails_the_call_then_recovers)
FAULT_LIB = os.path.join(LIBDIR, "libgpu_nnue_fault.so")
FAULT_DEFINES = ("-DGN_FAULT_PLAN_BLOCK=1",)
# test-only variant: eval_net<128>'s gather at an odd depth (5 rows in flight; the default is 4), so
# that the odd depth's last-row add and its tail are exercised (ADVICE r5;
# tests/test_gpu_parity.py::test_small_net_odd_gather_depth_vs_oracle)
ODD_LIB = os.path.join(LIBDIR, "libgpu_nnue_d5.so")
ODD_DEFINES = ("-DGN_SMALL_DEPTH=5",)
SOURCES = ["gpu_nnue.hip", "kernels.hip", "stream.hip"]
HEADERS = ["chess.h", "host_board.h", "nnue.h", "kernels.h", "sha256.h", "device_util.h", "archive.h"]
ARCH = "gfx950"


def source_hash(defines=()) -> str:
    """SHA-256 over every source and header the library is built from, and the flags."""
    import hashlib
    h = hashlib.sha256()
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "gpu_nnue.h")]
    for d in deps:
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(" ".join([ARCH, *defines]).encode())
    return h.hexdigest()


def _stale(lib: str, defines=()) -> bool:
    """The library is current when the hash stored beside it (<lib>.sha256, written by the build
    that produced it) equals the sources' hash: a copied tree (the gpurun snapshot) with other
    sources rebuilds, whatever the file times say."""
    stamp = lib + ".sha256"
    if not os.path.exists(lib) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != source_hash(defines)


def build(force: bool = False, verbose: bool = False, defines=(), out: str | None = None) -> str:
    """defines/out: experiment variants (e.g. -DGN_EXPAND_WPE=5 into lib/libgpu_nnue_w5.so),
    selected at run time with GPU_NNUE_LIB; the default build has neither."""
    lib = out or LIB
    if not force and not _stale(lib, defines):
        return lib
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
    with open(lib + ".sha256", "w") as f:
        f.write(source_hash(defines) + "\n")
    for o in objs:
        os.remove(o)
    return lib


def build_rev(rev: str, out: str, defines=()) -> str:
    """A/B baseline: the library as of git revision `rev` (its csrc/ and include/ extracted into a
    temporary tree), into lib/<out>.  Used on the CPU before an A/B run; never by the product."""
    import shutil
    import tempfile
    tmp = tempfile.mkdtemp(prefix="gn_rev_")
    try:
        arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "fishnet_amd/csrc", "include"],
                              check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
        objs = []
        for src in SOURCES:
            obj = os.path.join(tmp, src.replace(".hip", ".o"))
            subprocess.run(["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                            "-w", *defines, "-c", os.path.join(tmp, "fishnet_amd", "csrc", src), "-o", obj],
                           check=True)
            objs.append(obj)
        lib = os.path.join(LIBDIR, out)
        subprocess.run(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-lpthread"],
                       check=True)
        return lib
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def build_fault(force: bool = False, verbose: bool = False) -> str:
    """The fault-injection library (never loaded by the product path or the bench)."""
    return build(force=force, verbose=verbose, defines=FAULT_DEFINES, out=FAULT_LIB)


def build_odd(force: bool = False, verbose: bool = False) -> str:
    """The odd-gather-depth library (test only; never loaded by the product path or the bench)."""
    return build(force=force, verbose=verbose, defines=ODD_DEFINES, out=ODD_LIB)


DROPIN_NATIVE = os.path.join(LIBDIR, "dropin_native")


def build_dropin_native(force: bool = False) -> str:
    """tools/dropin_native.c (bench.py secondary.dropin's native 16-caller line) against the built
    library; rebuilt when the source or the library is newer than the binary."""
    lib = build()
    src = os.path.join(os.path.dirname(HERE), "tools", "dropin_native.c")
    out = DROPIN_NATIVE
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(src), os.path.getmtime(lib)):
        return out
    tmp = out + f".{os.getpid()}"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-Wall", "-o", tmp, src, f"-L{LIBDIR}", "-lgpu_nnue", "-lpthread",
                    "-Wl,-rpath,$ORIGIN", "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    outs = [a[len("--out="):] for a in sys.argv[1:] if a.startswith("--out=")]
    revs = [a[len("--rev="):] for a in sys.argv[1:] if a.startswith("--rev=")]
    if revs:
        print(build_rev(revs[0], outs[0] if outs else f"libgpu_nnue_{revs[0]}.so", defines=defs))
        sys.exit(0)
    print(build(force="--force" in sys.argv, verbose=True, defines=defs,
                out=os.path.join(LIBDIR, outs[0]) if outs else None))
