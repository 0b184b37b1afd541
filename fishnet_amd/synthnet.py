"""Seeded synthetic Stockfish-format .nnue networks (writer) + format helpers.

The real nets named by the reference (`nn-1c0000000000.nnue` big,
`nn-37f18f62d772.nnue` small; /root/reference/build.rs:8-9) are not in this
container and cannot be fetched (`make net` needs the network,
/root/reference/build.rs:318-333).  Benchmarks and parity tests therefore use
nets of identical shape and file format written here from a seed.

File layout written (Stockfish 17.1-era NNUE format):
  u32 version 0x7AF32F20 | u32 network hash | u32 len + description
  u32 FT hash | LEB128(int16 biases[L1]) | LEB128(int16 weights[22528][L1])
              | LEB128(int32 psqt[22528][8])
  8 x ( u32 arch hash | i32 b0[16] i8 w0[16][L1] | i32 b1[32] i8 w1[32][32]
        | i32 b2[1] i8 w2[1][32] )
All weights come from a counter-based splitmix64 stream mapped to an
Irwin-Hall approximate normal with integer arithmetic only, so the bytes are
identical on every machine and numpy version (tests pin a sha256).
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np

FT_INPUTS = 22528
PSQT_BUCKETS = 8
LAYER_STACKS = 8
VERSION = 0x7AF32F20
LEB_MAGIC = b"COMPRESSED_LEB128"
BIG_L1, SMALL_L1 = 3072, 128
M64 = (1 << 64) - 1


def _affine_hash(prev: int, outs: int) -> int:
    h = (0xCC03DAE4 + outs) & 0xFFFFFFFF
    h ^= prev >> 1
    h ^= (prev << 31) & 0xFFFFFFFF
    return h


def hashes(l1: int):
    """(network hash, FT hash, layer-stack hash) for an L1-wide net."""
    ft = 0x7F234CB8 ^ (l1 * 2)
    h = 0xEC42E90D ^ (l1 * 2)
    h = _affine_hash(h, 16)
    h = (0x538D24C7 + h) & 0xFFFFFFFF
    h = _affine_hash(h, 32)
    h = (0x538D24C7 + h) & 0xFFFFFFFF
    h = _affine_hash(h, 1)
    return ft ^ h, ft, h


def leb128_encode(vals: np.ndarray) -> bytes:
    """Signed LEB128 of every value (vectorised, chunked)."""
    out = []
    flat = np.asarray(vals).reshape(-1)
    for lo in range(0, flat.size, 1 << 22):
        v = flat[lo:lo + (1 << 22)].astype(np.int64)
        nb = np.ones(v.size, dtype=np.int64)
        for k in range(1, 6):
            lim = 1 << (7 * k - 1)
            nb += ((v < -lim) | (v >= lim)).astype(np.int64)
        buf = np.empty(int(nb.sum()), dtype=np.uint8)
        starts = np.cumsum(nb) - nb
        for k in range(int(nb.max())):
            m = nb > k
            byte = (v[m] >> (7 * k)) & 0x7F
            cont = (nb[m] > k + 1).astype(np.int64) << 7
            buf[starts[m] + k] = (byte | cont).astype(np.uint8)
        out.append(buf.tobytes())
    payload = b"".join(out)
    return LEB_MAGIC + struct.pack("<I", len(payload)) + payload


def leb128_decode(blob: bytes, count: int, bits: int) -> np.ndarray:
    """Reference-semantics decoder (slow path, used by tests on small blocks)."""
    assert blob[:17] == LEB_MAGIC
    (n,) = struct.unpack_from("<I", blob, 17)
    p, end = 21, 21 + n
    out = np.empty(count, dtype=np.int16 if bits == 16 else np.int32)
    for i in range(count):
        result, shift = 0, 0
        while True:
            byte = blob[p]
            p += 1
            result |= (byte & 0x7F) << shift
            shift += 7
            if not byte & 0x80:
                if byte & 0x40:
                    result -= 1 << shift
                break
        out[i] = ((result + (1 << (bits - 1))) % (1 << bits)) - (1 << (bits - 1))
    assert p == end
    return out


def _splitmix(seed: int, stream: int, lo: int, n: int) -> np.ndarray:
    i = np.arange(lo, lo + n, dtype=np.uint64) + np.uint64(1)
    base = np.uint64(((seed * 0x9E3779B97F4A7C15) + stream * 0xD1B54A32D192ED03) & M64)
    with np.errstate(over="ignore"):
        z = base + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _normal(seed: int, stream: int, n: int, sigma: float, mean: int = 0) -> np.ndarray:
    """Integer Irwin-Hall(4) approximate normal, exactly reproducible."""
    out = np.empty(n, dtype=np.int64)
    num = int(round(sigma * 1024))
    for lo in range(0, n, 1 << 22):
        k = min(1 << 22, n - lo)
        r = _splitmix(seed, stream, lo, k)
        s = np.zeros(k, dtype=np.int64)
        for j in range(4):
            s += ((r >> np.uint64(16 * j)) & np.uint64(0xFFFF)).astype(np.int64)
        out[lo:lo + k] = mean + ((s - 131070) * num) // (37837 * 1024)
    return out


def synth_net_arrays(l1: int, seed: int, stress: bool = False) -> dict:
    """The integer parameter arrays of a synthetic net, exactly as stored in
    the file (feature-transformer values NOT doubled)."""
    assert l1 % 32 == 0 and 32 <= l1 <= 4096
    ft_sigma = 6000.0 if stress else 18.0
    a = {
        "ft_bias": np.clip(_normal(seed, 1, l1, 60.0, 40), -16383, 16383).astype(np.int16),
        "ft_w": np.clip(_normal(seed, 2, FT_INPUTS * l1, ft_sigma), -16383, 16383).astype(np.int16)
        .reshape(FT_INPUTS, l1),
        "psqt": _normal(seed, 3, FT_INPUTS * PSQT_BUCKETS, 1000.0).astype(np.int32).reshape(FT_INPUTS, 8),
        "b0": [], "w0": [], "b1": [], "w1": [], "b2": [], "w2": [],
    }
    s0 = 200.0 / np.sqrt(l1)
    for b in range(LAYER_STACKS):
        st = 100 + 10 * b
        w0 = _normal(seed, st + 1, 16 * l1, s0).reshape(16, l1)
        w0 -= w0.sum(axis=1, keepdims=True) // l1  # ~zero-sum rows: inputs are >= 0
        w0[15] //= 4                                # keep the skip term modest
        a["b0"].append(_normal(seed, st + 0, 16, 1000.0).astype(np.int32))
        a["w0"].append(np.clip(w0, -128, 127).astype(np.int8))
        a["b1"].append(_normal(seed, st + 2, 32, 2000.0).astype(np.int32))
        a["w1"].append(np.clip(_normal(seed, st + 3, 32 * 32, 16.0), -128, 127).astype(np.int8).reshape(32, 32))
        a["b2"].append(_normal(seed, st + 4, 1, 300.0).astype(np.int32))
        a["w2"].append(np.clip(_normal(seed, st + 5, 32, 6.0), -128, 127).astype(np.int8))
    return a


def synth_net_bytes(l1: int, seed: int, stress: bool = False,
                    description: str | None = None) -> bytes:
    """A complete .nnue image for an L1-wide HalfKAv2_hm network.

    stress=True uses feature-transformer weights large enough that the int16
    accumulators wrap often (exercises the wrapping semantics)."""
    a = synth_net_arrays(l1, seed, stress)
    net_hash, ft_hash, arch_hash = hashes(l1)
    desc = (description or f"fishnet_amd synthetic net L1={l1} seed={seed} stress={int(stress)}").encode()
    parts = [struct.pack("<III", VERSION, net_hash, len(desc)), desc, struct.pack("<I", ft_hash),
             leb128_encode(a["ft_bias"]), leb128_encode(a["ft_w"]), leb128_encode(a["psqt"])]
    for b in range(LAYER_STACKS):
        parts += [struct.pack("<I", arch_hash)] + [a[k][b].astype("<i4" if k[0] == "b" else np.int8).tobytes()
                                                   for k in ("b0", "w0", "b1", "w1", "b2", "w2")]
    return b"".join(parts)


def write_synth_net(path: str, l1: int, seed: int, stress: bool = False) -> str:
    data = synth_net_bytes(l1, seed, stress)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)
    return hashlib.sha256(data).hexdigest()


def cached_synth_net(l1: int, seed: int, stress: bool = False, cache_dir: str | None = None) -> str:
    """Path of a synthetic net, generated once into a cache directory."""
    cache_dir = cache_dir or os.environ.get("GPU_NNUE_CACHE") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), ".cache")
    os.makedirs(cache_dir, exist_ok=True)
    path = os.path.join(cache_dir, f"synth_L{l1}_s{seed}{'_stress' if stress else ''}.nnue")
    if not os.path.exists(path):
        write_synth_net(path, l1, seed, stress)
    return path


def net_paths():
    """(big, small, label): real nets from GPU_NNUE_BIG / GPU_NNUE_SMALL if set,
    otherwise seeded synthetic nets of identical shape."""
    big, small = os.environ.get("GPU_NNUE_BIG"), os.environ.get("GPU_NNUE_SMALL")
    if big and small and os.path.exists(big) and os.path.exists(small):
        return big, small, "real"
    return cached_synth_net(BIG_L1, 1), cached_synth_net(SMALL_L1, 2), "synthetic(seed big=1 small=2)"
