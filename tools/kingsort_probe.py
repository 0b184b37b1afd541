"""Probe (timing only): does ordering the expansion's parents by king buckets raise the
stream's L2 hits?  The bench's 49,152 random 80-ply games, expanded (big net, incremental)
in game order and in orders sorted (stable) by the HalfKAv2_hm king buckets of the two
perspectives; chain 81 and chain 1.  Prints stream / plan ms and FT rows per variant."""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from fishnet_amd import gpu_nnue as G, synthnet  # noqa: E402


def king_squares(b):
    occ = b["occ"].astype(np.uint64)
    bits = ((occ[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    idx = np.cumsum(bits, axis=1) - 1                      # nibble index of each occupied square
    pc = np.frombuffer(b["pc"].tobytes(), dtype=np.uint8).reshape(len(b), 16)
    order = np.empty((len(b), 32), dtype=np.uint8)          # nibble k = byte k/2, low half first
    order[:, 0::2], order[:, 1::2] = pc & 15, pc >> 4
    piece = np.where(bits, np.take_along_axis(order, np.clip(idx, 0, 31), axis=1), 0)
    wk = np.argmax(piece == 6, axis=1)
    bk = np.argmax(piece == 14, axis=1)
    return wk, bk


def bucket(sq):
    f, r = sq & 7, sq >> 3
    return r * 4 + np.minimum(f, 7 - f)


def main():
    games, plies = int(sys.argv[1]) if len(sys.argv) > 1 else 49152, 80
    nn = G.GpuNnue(synthnet.cached_synth_net(3072, 1), synthnet.cached_synth_net(128, 2))
    n = games * (plies + 1)
    d_p = nn.alloc(n * 32)
    nn.random_games_device(0x5EED0000, 0, games, plies, d_p)
    nn.synchronize()
    b = d_p.download(G.BOARD_DTYPE, n)
    wk, bk = king_squares(b)
    bw, bb = bucket(wk), bucket(bk ^ 56)
    print("distinct bucket pairs", len(np.unique(bw * 32 + bb)), "top share",
          np.bincount(bw * 32 + bb, minlength=1024).max() / n, flush=True)
    orders = {"game": np.arange(n), "pair": np.argsort(bw * 32 + bb, kind="stable"),
              "white": np.argsort(bw, kind="stable")}
    res = {}
    for name, o in orders.items():
        d_p.upload(b[o])
        for chain in (81, 1):
            nn.set_option(G.OPT_CHAIN, chain)
            nn.time_expand_device(d_p, n, 1, 1)
            ms, t, st, rows = nn.time_expand_device(d_p, n, 1, 3)
            r = dict(ms=ms / 3, stream=nn.get_option(G.STAT_STREAM_NS) / 1e6,
                     plan=nn.get_option(G.STAT_PLAN_NS) / 1e6, rows=rows, children=t)
            res[f"{name}/{chain}"] = r
            print(name, chain, json.dumps(r), flush=True)
    nn.set_option(G.OPT_CHAIN, 81)


if __name__ == "__main__":
    main()
