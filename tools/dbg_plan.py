"""Debug: planned vs old expansion on a few FENs (prints mismatching parents / children)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from fishnet_amd import gpu_nnue as G, synthnet
from oracle import oracle as O
O.build()
bp, sp = synthnet.cached_synth_net(3072, 1), synthnet.cached_synth_net(128, 2)
ob, osm = O.Net(bp), O.Net(sp)
ctx = G.GpuNnue(bp, sp)
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
fens = [START, "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", START,
        "4k3/8/8/8/8/8/4P3/4K3 w - - 0 1"] + [G.board_to_fen(b) for b in G.random_positions(5, 0, 40, 160)]
for chain in (1, -2):
    ctx.set_option(G.OPT_CHAIN, chain)
    for mode in (1, 0):
        par, offs, mv, kids = ctx.expand_and_evaluate(fens, mode)
        bad = []
        for i, f in enumerate(fens):
            pe, me, ke = O.expand_eval(ob, osm, f, mode)
            got = dict(zip(mv[offs[i]:offs[i + 1]].tolist(), map(tuple, kids[offs[i]:offs[i + 1]].tolist())))
            exp = dict(zip(me, map(tuple, ke.tolist())))
            nb = sum(got.get(m) != exp[m] for m in exp)
            if tuple(par[i]) != pe or nb:
                bad.append((i, tuple(par[i]), pe, nb, len(exp)))
        print("stream", os.environ.get("GN_STREAM", "new"), "chain", chain, "mode", mode, "bad", len(bad), bad[:6], flush=True)
