"""Regenerates tests/golden/score_fens.json: positions for the score rule (gpu_nnue.h, gn_eval.score)
and the oracle's records for them.

The reference requires a score for every analysed position (/root/reference/src/stockfish.rs:366-368,
src/ipc.rs:56 `expect("got score")`), which Stockfish's search always prints; the static evaluation
has none in check.  The fixture holds positions of every branch of the rule, found by seeded random
games on the oracle's own movegen:
  mate0        checkmate (no legal move, in check)       -> mate 0
  stalemate    no legal move, not in check               -> cp 0
  searched_d1  in check, no reply in check               -> negamax over the replies' static values
  searched_d2  in check, some reply in check with moves  -> that reply is searched one level down
  mate+        in check, a reply mates                    -> mate 1 (and other positive mates)
  mate-        in check, every reply loses to a mate      -> mate -1
plus hand-written known cases (Fool's mate, the Opera game's final position, a queen stalemate).
Records (psqt, positional, final_v, final_cp, score, flags, best_move) are the CPU oracle's on the
seeded synthetic nets (sha256 pinned); self-consistency goldens, NOT Stockfish outputs.
Run from the repo root:  python tests/golden/make_score_fens.py
"""
import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from fishnet_amd import synthnet  # noqa: E402
from oracle import oracle as O  # noqa: E402

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
KNOWN = {
    "mate0": ["rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 1 3",  # Fool's mate
              "1n1Rkb1r/p4ppp/4q3/4p1B1/4P3/8/PPP2PPP/2K5 b k - 1 17"],      # Opera game, final position
    "stalemate": ["7k/5Q2/6K1/8/8/8/8/8 b - - 0 1"],
}
PER_CATEGORY = 12


def classify(small, fen, moves):
    e = O.eval_fen(None, small, fen, O.MODE_SMALL)
    fl = e[5]
    if fl & O.FLAG_NO_MOVES:
        return "mate0" if fl & O.FLAG_IN_CHECK else "stalemate"
    if not fl & O.FLAG_SEARCHED:
        return None
    if fl & O.FLAG_MATE:
        return "mate+" if e[4] > 0 else "mate-"
    for m in moves:
        c = O.eval_fen(None, small, O.child_fen(fen, m), O.MODE_SMALL)
        if c[5] & (O.FLAG_IN_CHECK | O.FLAG_NO_MOVES) == O.FLAG_IN_CHECK:
            return "searched_d2"
    return "searched_d1"


def find(small, seed=7, games=3000):
    rng, cats = random.Random(seed), {k: list(v) for k, v in KNOWN.items()}
    for _ in range(games):
        fen = START
        for _ in range(200):
            moves = O.legal_moves(fen)
            k = classify(small, fen, moves)
            if k and len(cats.setdefault(k, [])) < PER_CATEGORY and fen not in cats[k]:
                cats[k].append(fen)
            if not moves:
                break
            fen = O.child_fen(fen, rng.choice(moves))
    return cats


def main():
    big_p, small_p = synthnet.cached_synth_net(3072, 1), synthnet.cached_synth_net(128, 2)
    big, small = O.Net(big_p), O.Net(small_p)
    cats = find(small)
    fens = [f for k in sorted(cats) for f in cats[k]]
    sha = lambda p: hashlib.sha256(open(p, "rb").read()).hexdigest()
    res = {}
    for name, mode in (("full", 0), ("big", 1), ("small", 2)):
        out = O.eval_fens(big, small, fens, mode, threads=8)
        res[name] = [[f] + [int(x) for x in r] for f, r in zip(fens, out.tolist())]
    doc = {"_source": "CPU oracle (oracle/oracle.c) on seeded synthetic nets; positions from seeded random games "
                      "(tests/golden/make_score_fens.py); self-consistency goldens, NOT Stockfish outputs.",
           "nets": {"big": {"l1": 3072, "seed": 1, "sha256": sha(big_p)},
                    "small": {"l1": 128, "seed": 2, "sha256": sha(small_p)}},
           "categories": cats,
           "columns": ["fen", "psqt", "positional", "final_v", "final_cp", "score", "flags", "best_move"],
           "results": res}
    with open(os.path.join(ROOT, "tests", "golden", "score_fens.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print({k: len(v) for k, v in cats.items()})


if __name__ == "__main__":
    main()
