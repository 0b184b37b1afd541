#!/usr/bin/env python3
"""PCIe-inclusive rates of the host entry points: FEN text in host
memory -> parse -> H2D -> evaluation -> D2H -> gn_eval in host memory.  Not the
bench's `value` (that is HBM-resident); reported beside it.

  gn_evaluate_batch (mode FULL and BIG) over N random-playout FENs;
  gn_expand_and_evaluate over the consecutive positions of G random 80-ply games
  (every position + every legal child; the chained walk and king cache engage).
Prints one JSON line.  Usage: python tools/host_path.py [--fens N] [--games G]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fens", type=int, default=1 << 20)
    ap.add_argument("--games", type=int, default=2048)
    args = ap.parse_args()
    from fishnet_amd import gpu_nnue as G, synthnet
    big, small, label = synthnet.net_paths()
    nn = G.GpuNnue(big, small, devices=[0])
    out = {"nets": label}
    boards = G.random_positions(0x5EED0000, 0, args.fens, 160)
    fens = [G.board_to_fen(b) for b in boards]
    import numpy as np
    arr, _keep = G._fen_array(fens)  # the char* array a caller holds (not timed)
    res = np.zeros(len(fens), dtype=G.EVAL_DTYPE)
    for mode, name in ((G.MODE_FULL, "full"), (G.MODE_BIG, "big")):
        nn.evaluate_batch(fens[:4096], mode)  # warm-up (allocations)
        t = time.perf_counter()
        G._check(G.lib().gn_evaluate_batch_mode(nn.h, arr, len(fens), mode, res.ctypes.data))
        dt = time.perf_counter() - t
        out[f"evaluate_batch_{name}"] = {"fens": len(fens), "s": round(dt, 3), "evals_per_s": round(len(fens) / dt)}
    plies = 80
    n = args.games * (plies + 1)
    d = nn.alloc(n * 32)
    nn.random_games_device(0x5EED0000, 0, args.games, plies, d)
    nn.synchronize()
    gfens = [G.board_to_fen(b) for b in d.download(G.BOARD_DTYPE, n)]
    nn.expand_and_evaluate(gfens[:810], G.MODE_FULL)
    t = time.perf_counter()
    parents, offs, moves, kids = nn.expand_and_evaluate(gfens, G.MODE_FULL, cap=64 * n)
    dt = time.perf_counter() - t
    ev = len(parents) + len(kids)
    out["expand_and_evaluate_full"] = {"games": args.games, "parents": len(parents), "children": len(kids),
                                       "s": round(dt, 3), "evals_per_s": round(ev / dt)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
