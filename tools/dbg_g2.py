"""Debug: depth-2 grandchildren vs the plain depth-1 path, mode FULL (which side is wrong)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: F401
from fishnet_amd import gpu_nnue as G, synthnet
from oracle import oracle as O
from test_gpu_parity import special_fens, _expand2

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
big_p, small_p = synthnet.cached_synth_net(3072, 1), synthnet.cached_synth_net(128, 2)
ctx = G.GpuNnue(big_p, small_p, devices=[0])
ob, osm = O.Net(big_p), O.Net(small_p)
games, plies = 3, 80
n0 = games * (plies + 1)
d_g = ctx.alloc(n0 * 32)
ctx.random_games_device(0x5EED0077, 0, games, plies, d_g)
ctx.synchronize()
boards = np.concatenate([d_g.download(G.BOARD_DTYPE, n0), G.pack_fens(special_fens())[0]])
n = len(boards)
d_b = ctx.alloc(n * 32)
d_b.upload(boards)
for opts in ((81, 1), (81, 0), (1, 1)):
    ctx.set_option(G.OPT_CHAIN, opts[0]); ctx.set_option(G.OPT_KING_CACHE, opts[1])
    t, g, out = _expand2(ctx, d_b, n, mode)
    gco = out["gco"].download(G.EVAL_DTYPE, g)
    goff = out["goff"].download(np.uint32, t + 1)
    gmv = out["gmv"].download(np.uint16, g)
    kids = out["ch"].download(G.BOARD_DTYPE, t)
    ctx.set_option(G.OPT_CHAIN, 1); ctx.set_option(G.OPT_KING_CACHE, 0)
    b2 = {k: ctx.alloc(sz) for k, sz in (("po", t * 16), ("off", (t + 1) * 4), ("ch", g * 32), ("mv", g * 2), ("co", g * 16))}
    ctx.expand_device(out["ch"], t, mode, b2["po"], b2["off"], b2["ch"], b2["mv"], b2["co"], g)
    pco = b2["co"].download(G.EVAL_DTYPE, g)
    bad = np.nonzero(gco != pco)[0]
    par = np.searchsorted(goff, bad, side="right") - 1
    print("opts", opts, "t", t, "g", g, "bad grandchildren", len(bad), "distinct children", len(np.unique(par)), flush=True)
    for j in np.unique(par)[:6]:
        lo, hi = int(goff[j]), int(goff[j + 1])
        fen = G.board_to_fen(kids[j])
        p_exp, m_exp, k_exp = O.expand_eval(ob, osm, fen, mode, incremental=True)
        exp = dict(zip(m_exp, map(tuple, k_exp.tolist())))
        e2 = sum(tuple(gco[i]) != exp[int(gmv[i])] for i in range(lo, hi))
        pl = sum(tuple(pco[i]) != exp[int(gmv[i])] for i in range(lo, hi))
        print("  child", j, "kids", hi - lo, "bad in expand2", e2, "bad in plain", pl, fen, flush=True)
    for b in b2.values(): b.free()
ctx.close()
