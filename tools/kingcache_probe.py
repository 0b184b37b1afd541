"""CPU probe: FT rows per position of configs[2] (big-net full refresh of
unrelated random-playout positions) if each king-sorted position were refreshed from the block's
king cache -- Stockfish's AccumulatorCaches: the accumulator last computed in the block for the
same perspective and king square, plus the placement difference -- instead of eval_net<3072>'s
bias + common-row base + per-position rows (33.7 rows per position, profiles/r05z).

Positions: the bench's big16m generator (gn_random_positions, seed SEED, <= 160 plies) on the
host; order: the library's king-sort key (king_keys_kernel: white king, black king, layer-stack
bucket, 30 home-square bits); blocks of K consecutive sorted positions, cache cold at each block
start (plan_kernel's per-block cache).  Rows of perspective h at position i: 1 + P when the
block holds no earlier position with h's king on the same square, else 1 + min(P, d) with d the
placement difference (a square whose piece changed counts 2: remove + add).

    python tools/kingcache_probe.py [n_positions] [K]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from fishnet_amd import gpu_nnue as G  # noqa: E402

SEED = 0x5EED0000


def pieces(b):
    occ = b["occ"].astype(np.uint64)
    bits = ((occ[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    idx = np.cumsum(bits, axis=1) - 1
    pc = np.frombuffer(b["pc"].tobytes(), dtype=np.uint8).reshape(len(b), 16)
    nib = np.empty((len(b), 32), dtype=np.uint8)
    nib[:, 0::2], nib[:, 1::2] = pc & 15, pc >> 4
    return np.where(bits, np.take_along_axis(nib, np.clip(idx, 0, 31), axis=1), 0).astype(np.uint8)


def sort_keys(pl):
    n = len(pl)
    wk, bk = np.argmax(pl == 6, axis=1).astype(np.uint64), np.argmax(pl == 14, axis=1).astype(np.uint64)
    cnt = (pl != 0).sum(axis=1)
    b = ((cnt - 1) // 4).astype(np.uint64)
    back = [4, 2, 3, 5, 6, 3, 2, 4]  # ROOK KNIGHT BISHOP QUEEN KING BISHOP KNIGHT ROOK (white codes)
    want = np.full(64, 255, dtype=np.int32)
    for f in range(8):
        want[f], want[8 + f], want[48 + f], want[56 + f] = back[f], 1, 9, 8 + back[f]
    home = (pl == want[None, :])
    sq = [s for s in range(16) if s != 4] + [s for s in range(48, 64) if s != 60]
    r = np.zeros(n, dtype=np.uint64)
    for s in sq:  # lowest square most significant
        r = (r << np.uint64(1)) | home[:, s].astype(np.uint64)
    return (wk << np.uint64(58)) | (bk << np.uint64(52)) | (b << np.uint64(49)) | (r << np.uint64(19)), wk, bk


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 81
    b = G.random_positions(SEED, 0, n, 160)
    pl = pieces(b)
    key, wk, bk = sort_keys(pl)
    order = np.argsort(key, kind="stable")
    pl, wk, bk = pl[order], wk[order].astype(np.int64), bk[order].astype(np.int64)
    P = (pl != 0).sum(axis=1)
    blk = np.arange(n) // K
    total = np.zeros(n, dtype=np.int64)
    hits = 0
    for ks in (wk, bk):
        # the previous position of the block with this perspective's king on the same square
        g = np.lexsort((np.arange(n), ks, blk))
        same = np.zeros(n, dtype=bool)
        same[1:] = (blk[g][1:] == blk[g][:-1]) & (ks[g][1:] == ks[g][:-1])
        prev = np.full(n, -1, dtype=np.int64)
        prev[g[1:][same[1:]]] = g[:-1][same[1:]]
        has = prev >= 0
        a, c = pl[has], pl[prev[has]]
        d = ((a != c) & (a != 0)).sum(axis=1) + ((a != c) & (c != 0)).sum(axis=1)
        rows = 1 + P.copy()
        rows[has] = 1 + np.minimum(P[has], d)
        hits += int((has & (rows < 1 + P)).sum())
        total += rows
    print(f"n={n} K={K}: rows per position {total.mean():.2f} (full refresh 2 * (1 + P) = {2 * (1 + P.mean()):.2f}); "
          f"king-cache hits {hits / (2 * n):.3f} of refreshes; mean pieces {P.mean():.2f}")


if __name__ == "__main__":
    main()
