"""GPU parity: libgpu_nnue (HIP, gfx950) against the CPU oracle, bit-exact.

Every check here compares integers, so the bar is exact equality (north star:
"Results must match ... bit-exactly, since all arithmetic is integer").
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def special_fens():
    with open(os.path.join(HERE, "golden", "special_fens.txt")) as f:
        return [l.strip() for l in f if l.strip() and not l.startswith("#")]


def random_fens(n, seed, max_plies=160):
    from fishnet_amd import gpu_nnue as G
    boards = G.random_positions(seed, 0, n, max_plies)
    return [G.board_to_fen(b) for b in boards]


STATIC = ["psqt", "positional", "final_v", "final_cp"]


def static_part(rec):
    """The static evaluation of a record (a child record and the same position's scored record
    agree on it; the score fields differ by design, gpu_nnue.h at gn_eval)."""
    r = np.asarray(rec)
    return [tuple(int(x) for x in t) for t in r[STATIC].tolist()], (r["flags"] & 15).tolist()


def _cmp(got, exp, fens):
    bad = np.nonzero(got != exp)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{len(bad)} mismatches; first {fens[i]!r}: gpu={got[i]} oracle={exp[i]}")


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_special_fens_all_modes(gpu_ctx, oracle_nets, oracle_lib, mode):
    big, small = oracle_nets
    fens = special_fens()
    _cmp(gpu_ctx.evaluate_batch(fens, mode), oracle_lib.eval_fens(big, small, fens, mode, threads=8), fens)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_random_playouts_all_modes(gpu_ctx, oracle_nets, oracle_lib, mode):
    big, small = oracle_nets
    fens = random_fens(3000, 0x5EED0000 + 17 * mode)
    got = gpu_ctx.evaluate_batch(fens, mode)
    _cmp(got, oracle_lib.eval_fens(big, small, fens, mode, threads=8), fens)
    if mode == 0:  # the FULL pipeline exercised every branch
        flags = got["flags"]
        assert (flags & 2).any() and (flags & 8).any() and ((flags & 10) == 0).any()


def test_golden_vectors(gpu_ctx):
    """The committed oracle goldens (tests/golden/eval_goldens.json) on the GPU."""
    g = json.load(open(os.path.join(HERE, "golden", "eval_goldens.json")))
    for mode_name, rows in g["results"].items():
        mode = {"full": 0, "big": 1, "small": 2}[mode_name]
        fens = [r[0] for r in rows]
        exp = np.array([tuple(r[1:]) for r in rows], dtype=gpu_ctx.evaluate_batch([], mode).dtype)
        _cmp(gpu_ctx.evaluate_batch(fens, mode), exp, fens)


def test_score_fixture_all_modes(gpu_ctx, oracle_nets, oracle_lib):
    """The score rule (gpu_nnue.h at gn_eval) on checkmates, stalemates and in-check positions
    whose replies are static, in check (searched one level down) or mating / mated: the
    committed oracle records, the live oracle, and the same positions as expansion parents."""
    from fishnet_amd import gpu_nnue as G
    g = json.load(open(os.path.join(HERE, "golden", "score_fens.json")))
    big, small = oracle_nets
    for name, mode in (("full", 0), ("big", 1), ("small", 2)):
        rows = g["results"][name]
        fens = [r[0] for r in rows]
        exp = np.array([tuple(r[1:]) for r in rows], dtype=G.EVAL_DTYPE)
        _cmp(oracle_lib.eval_fens(big, small, fens, mode), exp, fens)
        _cmp(gpu_ctx.evaluate_batch(fens, mode), exp, fens)
        parents, offs, moves, kids = gpu_ctx.expand_and_evaluate(fens, mode)
        _cmp(parents, exp, fens)
        assert (kids["flags"] & G.FLAG_NO_SCORE).all()  # (a gn_child carries no score)
        searched = (exp["flags"] & G.FLAG_SEARCHED) != 0
        assert searched.sum() >= 30 and (exp["flags"] & G.FLAG_NO_MOVES != 0).sum() >= 20
    d_b, d_o = gpu_ctx.alloc(len(fens) * 32), gpu_ctx.alloc(len(fens) * G.EVAL_SIZE)
    d_b.upload(G.pack_fens(fens)[0])
    gpu_ctx.evaluate_device(d_b, len(fens), 2, d_o)  # the device API runs the rule too
    _cmp(d_o.download(G.EVAL_DTYPE, len(fens)), exp, fens)


def test_bad_fens_flagged(gpu_ctx):
    fens = ["", "garbage", "8/8/8/8/8/8/8/8 w - - 0 1", "K7/8/8/8/8/8/8/7K w - - 0 1",
            "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", "P3k3/8/8/8/8/8/8/4K3 w - - 0 1",
            "4k3/8/8/8/8/8/8/R3K3 b - - 0 1x", "4k3/4R3/8/8/8/8/8/4K3 w - - 0 1"]
    out = gpu_ctx.evaluate_batch(fens, 0)
    assert [bool(f & 4) for f in out["flags"]] == [True, True, True, True, False, True, False, True]
    assert (out[out["flags"] & 4 != 0][["psqt", "positional", "final_v"]].tolist()
            == [(0, 0, 0)] * 6)


def test_stress_net_wraps(oracle_lib):
    """FT weights large enough that the int16 accumulators wrap constantly."""
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(128, 7, stress=True)
    ctx = G.GpuNnue(None, p)
    on = oracle_lib.Net(p)
    fens = special_fens() + random_fens(2000, 99)
    acc, _ = oracle_lib.accumulate(on, fens[2], 0)
    _cmp(ctx.evaluate_batch(fens, 2), oracle_lib.eval_fens(None, on, fens, 2, threads=8), fens)
    # sanity: the wrap really happens (|x2 accumulator| > 32767 before wrapping)
    assert np.abs(acc.astype(np.int32)).max() > 8000


def test_big_stress_net(oracle_lib):
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(3072, 11, stress=True)
    ctx = G.GpuNnue(p, None)
    on = oracle_lib.Net(p)
    fens = special_fens() + random_fens(500, 1234)
    _cmp(ctx.evaluate_batch(fens, 1), oracle_lib.eval_fens(on, None, fens, 1, threads=8), fens)


def test_big_stress_net_expansion(oracle_lib):
    """Big-net incremental children (the planned expansion) under constant int16 wrapping."""
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(3072, 11, stress=True)
    ctx = G.GpuNnue(p, None)
    on = oracle_lib.Net(p)
    fens = special_fens() + random_fens(60, 4343)
    parents, offs, moves, kids = ctx.expand_and_evaluate(fens, 1)
    for i, fen in enumerate(fens):
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(on, None, fen, 1)
        assert tuple(parents[i]) == p_exp, fen
        got = {int(m): tuple(k) for m, k in zip(moves[offs[i]:offs[i + 1]], kids[offs[i]:offs[i + 1]])}
        assert got == {int(m): tuple(k) for m, k in zip(m_exp, G.children_from_evals(k_exp))}, fen


def test_big_stress_net_chained_king_cache():
    """Chained walk + king cache under constant int16 wrapping: identical to one
    refresh-started workgroup per parent on whole random games."""
    from fishnet_amd import gpu_nnue as G, synthnet
    ctx = G.GpuNnue(synthnet.cached_synth_net(3072, 11, stress=True), None)
    games, plies = 24, 80
    n = games * (plies + 1)
    d_b = ctx.alloc(n * 32)
    ctx.random_games_device(0x5EED0000 + 99, 0, games, plies, d_b)
    ctx.synchronize()
    cap = 60 * n
    bufs = {k: ctx.alloc(sz) for k, sz in (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("ch", cap * 32),
                                              ("mv", cap * 2), ("co", cap * G.EVAL_SIZE))}

    def run(k, kc):
        ctx.set_option(G.OPT_CHAIN, k)
        ctx.set_option(G.OPT_KING_CACHE, kc)
        t = ctx.expand_device(d_b, n, 1, bufs["po"], bufs["off"], bufs["ch"], bufs["mv"], bufs["co"], cap)
        return bufs["po"].download(G.EVAL_DTYPE, n), bufs["co"].download(G.EVAL_DTYPE, t)

    ref = run(1, 0)
    for k, kc in ((-81, 1), (-81, 0), (-5, 1)):
        got = run(k, kc)
        assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1]), (k, kc)
    ctx.close()


def test_device_api_matches_host_api(gpu_ctx):
    from fishnet_amd import gpu_nnue as G
    boards = G.random_positions(42, 1000, 4099, 160)
    fens = [G.board_to_fen(b) for b in boards]
    d_b = gpu_ctx.alloc(boards.nbytes)
    d_o = gpu_ctx.alloc(len(boards) * G.EVAL_SIZE)
    d_b.upload(boards)
    for mode in (0, 1, 2):
        gpu_ctx.evaluate_device(d_b, len(boards), mode, d_o)
        gpu_ctx.synchronize()
        got = d_o.download(G.EVAL_DTYPE, len(boards))
        assert np.array_equal(got, gpu_ctx.evaluate_batch(fens, mode))
    ms, per = gpu_ctx.time_evaluate_device(d_b, len(boards), 1, d_o, 3)
    assert ms > 0 and per[2] > 0


def test_perft_known_answers(gpu_ctx):
    g = json.load(open(os.path.join(HERE, "golden", "perft.json")))
    for c in g["cases"]:
        for d, nodes in enumerate(c["nodes"], start=1):
            if nodes > 200_000_000:
                break
            assert gpu_ctx.perft(c["fen"], d) == nodes, (c["name"], d)


def test_perft_special_vs_oracle(gpu_ctx, oracle_lib):
    for fen in special_fens():
        for d in (1, 2, 3):
            assert gpu_ctx.perft(fen, d) == oracle_lib.perft(fen, d), (fen, d)


@pytest.mark.parametrize("incremental", [1, 0])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_expand_vs_oracle(gpu_ctx, oracle_nets, oracle_lib, mode, incremental):
    from fishnet_amd.gpu_nnue import OPT_INCREMENTAL_CHILDREN, children_from_evals, move_to_uci
    big, small = oracle_nets
    fens = special_fens() + random_fens(150, 777 + mode)
    gpu_ctx.set_option(OPT_INCREMENTAL_CHILDREN, incremental)
    try:
        parents, offs, moves, kids = gpu_ctx.expand_and_evaluate(fens, mode)
    finally:
        gpu_ctx.set_option(OPT_INCREMENTAL_CHILDREN, 1)
    for i, fen in enumerate(fens):
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, mode)
        assert tuple(parents[i]) == p_exp, fen
        lo, hi = int(offs[i]), int(offs[i + 1])
        got = {int(m): tuple(k) for m, k in zip(moves[lo:hi], kids[lo:hi])}
        exp = {int(m): tuple(k) for m, k in zip(m_exp, children_from_evals(k_exp))}
        assert set(got) == set(exp), (fen, sorted(map(move_to_uci, set(got) ^ set(exp))))
        bad = [move_to_uci(m) for m in got if got[m] != exp[m]]
        assert not bad, (fen, bad[:5])


def test_incremental_stress_wrap(oracle_lib):
    """Incremental deltas under constant int16 wrapping equal full refreshes."""
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(128, 7, stress=True)
    ctx = G.GpuNnue(None, p)
    on = oracle_lib.Net(p)
    fens = special_fens() + random_fens(100, 4242)
    parents, offs, moves, kids = ctx.expand_and_evaluate(fens, 2)
    for i, fen in enumerate(fens):
        _, m_exp, k_exp = oracle_lib.expand_eval(None, on, fen, 2)
        got = {int(m): tuple(k) for m, k in zip(moves[offs[i]:offs[i + 1]], kids[offs[i]:offs[i + 1]])}
        assert got == {int(m): tuple(k) for m, k in zip(m_exp, G.children_from_evals(k_exp))}, fen


def test_expand_device_matches_host(gpu_ctx):
    from fishnet_amd import gpu_nnue as G
    boards = G.random_positions(99, 0, 300, 160)
    fens = [G.board_to_fen(b) for b in boards]
    hp, hoffs, hmoves, hkids = gpu_ctx.expand_and_evaluate(fens, 0)
    n, cap = len(boards), int(hoffs[-1])
    bufs = {k: gpu_ctx.alloc(sz) for k, sz in (("b", n * 32), ("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4),
                                                  ("ch", cap * 32), ("mv", cap * 2), ("co", cap * G.EVAL_SIZE))}
    bufs["b"].upload(boards)
    total = gpu_ctx.expand_device(bufs["b"], n, 0, bufs["po"], bufs["off"], bufs["ch"], bufs["mv"], bufs["co"], cap)
    assert total == cap
    assert np.array_equal(bufs["off"].download(np.uint32, n + 1), hoffs)
    assert np.array_equal(bufs["mv"].download(np.uint16, cap), hmoves)
    assert np.array_equal(G.children_from_evals(bufs["co"].download(G.EVAL_DTYPE, cap)), hkids)
    assert np.array_equal(bufs["po"].download(G.EVAL_DTYPE, n), hp)
    kids = bufs["ch"].download(G.BOARD_DTYPE, 40)
    assert [G.board_to_fen(k) for k in kids[:3]]
    with pytest.raises(G.GnError):
        gpu_ctx.expand_device(bufs["b"], n, 0, bufs["po"], bufs["off"], bufs["ch"], bufs["mv"], bufs["co"], cap - 1)


def test_random_games_are_legal_lines(gpu_ctx, oracle_lib):
    from fishnet_amd import gpu_nnue as G
    games, plies = 24, 40
    d = gpu_ctx.alloc(games * (plies + 1) * 32)
    gpu_ctx.random_games_device(7, 0, games, plies, d)
    gpu_ctx.synchronize()
    b = d.download(G.BOARD_DTYPE, games * (plies + 1)).reshape(games, plies + 1)
    for g in range(games):
        fens = [G.board_to_fen(x) for x in b[g]]
        assert fens[0].startswith("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq")
        for a, c in zip(fens, fens[1:]):
            if a == c:
                assert not oracle_lib.legal_moves(a) or int(a.split()[4]) >= 100
                continue
            kids = {oracle_lib.child_fen(a, m) for m in oracle_lib.legal_moves(a)}
            assert c in kids, (a, c)


def test_device_playouts_equal_host_playouts(gpu_ctx):
    from fishnet_amd import gpu_nnue as G
    host = G.random_positions(0x5EED0000, 12345, 500, 160)
    d = gpu_ctx.alloc(500 * 32)
    gpu_ctx.random_positions_device(0x5EED0000, 12345, 500, 160, d)
    gpu_ctx.synchronize()
    assert d.download(G.BOARD_DTYPE, 500).tobytes() == host.tobytes()


@pytest.mark.parametrize("swz,ksort", [(0, 0), (7, 0), (0, 1), (7, 1)])
def test_locality_options_do_not_change_results(gpu_ctx, swz, ksort):
    from fishnet_amd import gpu_nnue as G
    boards = G.random_positions(3, 0, 5003, 160)
    boards[17] = np.zeros(1, dtype=G.BOARD_DTYPE)  # an invalid board mixed in
    d_b, d_o = gpu_ctx.alloc(boards.nbytes), gpu_ctx.alloc(len(boards) * G.EVAL_SIZE)
    d_b.upload(boards)
    ref = {}
    for mode in (0, 1, 2):
        gpu_ctx.set_option(G.OPT_XCD_SWIZZLE, 0)
        gpu_ctx.set_option(G.OPT_KING_SORT, 0)
        gpu_ctx.evaluate_device(d_b, len(boards), mode, d_o)
        ref[mode] = d_o.download(G.EVAL_DTYPE, len(boards))
    try:
        gpu_ctx.set_option(G.OPT_XCD_SWIZZLE, swz)
        gpu_ctx.set_option(G.OPT_KING_SORT, ksort)
        for mode in (0, 1, 2):
            gpu_ctx.evaluate_device(d_b, len(boards), mode, d_o)
            assert np.array_equal(d_o.download(G.EVAL_DTYPE, len(boards)), ref[mode])
        assert ref[0][17]["flags"] & G.FLAG_BAD_FEN
        fens = [G.board_to_fen(b) for b in boards[:200] if b["occ"]]
        _, offs, moves, kids = gpu_ctx.expand_and_evaluate(fens, 1)
        gpu_ctx.set_option(G.OPT_XCD_SWIZZLE, 7 - swz)
        _, offs2, moves2, kids2 = gpu_ctx.expand_and_evaluate(fens, 1)
        assert np.array_equal(kids, kids2) and np.array_equal(moves, moves2)
        gpu_ctx.set_option(G.OPT_XCD_SWIZZLE, 8)  # XCD-local block claiming
        _, offs3, moves3, kids3 = gpu_ctx.expand_and_evaluate(fens, 1)
        assert np.array_equal(kids, kids3) and np.array_equal(moves, moves3)
    finally:
        gpu_ctx.set_option(G.OPT_XCD_SWIZZLE, 9)
        gpu_ctx.set_option(G.OPT_KING_SORT, 1)


@pytest.mark.parametrize("mode", [1, 0])
def test_chained_walk_matches_refresh_and_oracle(gpu_ctx, oracle_nets, oracle_lib, mode):
    """Chained walk (GN_OPT_CHAIN): consecutive game positions start from the previous
    parent's child accumulators, king-move children from the block's king cache
    (GN_OPT_KING_CACHE).  Every block length, with and without the cache, gives the
    refresh results, and the first games agree with the oracle."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 40, 80
    n = games * (plies + 1)
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0000, 0, games, plies, d_b)
    gpu_ctx.synchronize()
    boards = d_b.download(G.BOARD_DTYPE, n)
    cap = 60 * n
    bufs = {k: gpu_ctx.alloc(sz) for k, sz in (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("ch", cap * 32),
                                                  ("mv", cap * 2), ("co", cap * G.EVAL_SIZE))}

    def run(k):
        gpu_ctx.set_option(G.OPT_CHAIN, k)
        t = gpu_ctx.expand_device(d_b, n, mode, bufs["po"], bufs["off"], bufs["ch"], bufs["mv"], bufs["co"], cap)
        return (bufs["po"].download(G.EVAL_DTYPE, n), bufs["off"].download(np.uint32, n + 1),
                bufs["mv"].download(np.uint16, t), bufs["co"].download(G.EVAL_DTYPE, t))

    try:
        ref = run(1)
        for kc in (1, 0):
            gpu_ctx.set_option(G.OPT_KING_CACHE, kc)
            for k in (-81, -7, -2, 81):
                got = run(k)
                for a, b in zip(ref, got):
                    assert np.array_equal(a, b), (k, kc)
    finally:
        gpu_ctx.set_option(G.OPT_CHAIN, 81)
        gpu_ctx.set_option(G.OPT_KING_CACHE, 1)
    big, small = oracle_nets
    parents, offs, moves, kids = ref
    for i in range(2 * (plies + 1)):
        fen = G.board_to_fen(boards[i])
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, mode)
        assert tuple(parents[i]) == p_exp, fen
        lo, hi = int(offs[i]), int(offs[i + 1])
        got = {int(m): tuple(x) for m, x in zip(moves[lo:hi], kids[lo:hi])}
        assert got == {int(m): tuple(x) for m, x in zip(m_exp, k_exp)}, fen


@pytest.mark.parametrize("ksort", [2, 0])
def test_common_row_base_tiles(gpu_ctx, oracle_nets, oracle_lib, ksort):
    """eval_net's common-row base (pieces on the same square in every position of a
    16-position tile are gathered once per tile): consecutive positions of games share
    most pieces and alternate the side to move; runs of one repeated position make the
    whole placement common (zero per-position rows); invalid boards and a tile whose
    first position is invalid must not constrain the base.  Bit-exact vs the oracle,
    with the batch king/placement-sorted and in input order."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 12, 60
    n = games * (plies + 1)
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0077, 0, games, plies, d_b)
    gpu_ctx.synchronize()
    boards = d_b.download(G.BOARD_DTYPE, n)
    boards = np.concatenate([boards, np.repeat(boards[5:6], 40), np.repeat(boards[70:71], 17)])
    boards[32] = np.zeros(1, dtype=G.BOARD_DTYPE)  # first slot of a tile in input order
    boards[100] = np.zeros(1, dtype=G.BOARD_DTYPE)
    fens = [G.board_to_fen(b) if b["occ"] else "8/8/8/8/8/8/8/8 w - - 0 1" for b in boards]
    big, small = oracle_nets
    try:
        gpu_ctx.set_option(G.OPT_KING_SORT, ksort)
        for mode in (1, 0):
            got = gpu_ctx.evaluate_batch(fens, mode)
            ok = boards["occ"] != 0
            vf = [f for f, v in zip(fens, ok) if v]
            _cmp(got[ok], oracle_lib.eval_fens(big, small, vf, mode, threads=8), vf)
            assert got[32]["flags"] & G.FLAG_BAD_FEN and got[100]["flags"] & G.FLAG_BAD_FEN
    finally:
        gpu_ctx.set_option(G.OPT_KING_SORT, 1)


def test_chained_walk_at_bench_scale(gpu_ctx, oracle_nets, oracle_lib):
    """The chained walk + king cache at more than 2 x CARRY_SLOTS (2,048) blocks, so carry and
    king-cache slots are handed between workgroups and reused: 4,200 whole 80-ply games
    (340,200 parents, ~10 M children) against the plain path (one workgroup per parent,
    every parent refreshed, no king cache) by device checksums of every output, and 240
    sampled parents with all their children against the oracle."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 4200, 80
    n = games * (plies + 1)
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0000 + 4200, 0, games, plies, d_b)
    gpu_ctx.synchronize()
    _, total, _, _ = gpu_ctx.time_expand_device(d_b, n, 1, 1)
    out = {"po": gpu_ctx.alloc(n * G.EVAL_SIZE), "off": gpu_ctx.alloc((n + 1) * 4), "mv": gpu_ctx.alloc(total * 2),
           "co": gpu_ctx.alloc(total * G.EVAL_SIZE), "cap": total}

    def run(k, kc):
        gpu_ctx.set_option(G.OPT_CHAIN, k)
        gpu_ctx.set_option(G.OPT_KING_CACHE, kc)
        _, t, _, rows = gpu_ctx.time_expand_device(d_b, n, 1, 1, outputs=out)
        assert t == total
        return tuple(gpu_ctx.checksum_device(out[b], nb) for b, nb in
                     (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("mv", t * 2), ("co", t * G.EVAL_SIZE))), rows

    try:
        plain, rows_plain = run(1, 0)
        for k, kc in ((-81, 1), (81, 1), (-27, 1), (-81, 0)):
            got, rows = run(k, kc)
            assert got == plain, (k, kc)
            assert rows < rows_plain, (k, kc, rows, rows_plain)  # the chain / cache really engaged
        got, _ = run(81, 1)  # leave the default configuration's outputs in the buffers
    finally:
        gpu_ctx.set_option(G.OPT_CHAIN, 81)
        gpu_ctx.set_option(G.OPT_KING_CACHE, 1)
    big, small = oracle_nets
    boards = d_b.download(G.BOARD_DTYPE, n)
    offs = out["off"].download(np.uint32, n + 1)
    pev = out["po"].download(G.EVAL_DTYPE, n)
    rng = np.random.default_rng(7)
    idx = np.concatenate([rng.choice(n, 200, replace=False), np.arange(n - 40, n)])  # + the end of the last game
    for i in idx:
        fen = G.board_to_fen(boards[i])
        lo, hi = int(offs[i]), int(offs[i + 1])
        mv = out["mv"].download(np.uint16, hi - lo, offset=lo)
        ev = out["co"].download(G.EVAL_DTYPE, hi - lo, offset=lo)
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, 1, incremental=True)
        assert tuple(pev[i]) == p_exp, fen
        assert dict(zip(mv.tolist(), map(tuple, ev.tolist()))) == dict(zip(m_exp, map(tuple, k_exp.tolist()))), fen


def test_small_net_one_million_vs_oracle(gpu_ctx, oracle_nets, oracle_lib):
    """configs[1] at its full size: 1,048,576 random-playout positions, small net, bit-exact
    against the multithreaded oracle."""
    from fishnet_amd import gpu_nnue as G
    n = 1 << 20
    d_b, d_o = gpu_ctx.alloc(n * 32), gpu_ctx.alloc(n * G.EVAL_SIZE)
    gpu_ctx.random_positions_device(0x5EED0000, 0, n, 160, d_b)
    gpu_ctx.evaluate_device(d_b, n, G.MODE_SMALL, d_o)
    gpu_ctx.synchronize()
    got = d_o.download(G.EVAL_DTYPE, n)
    fens = G.boards_to_fens(d_b.download(G.BOARD_DTYPE, n))
    _, small = oracle_nets
    exp = oracle_lib.eval_fens(None, small, fens, 2, threads=16)
    _cmp(got, exp, fens)


def test_two_device_slots_shard_expansion_and_games(synth_big_path, synth_small_path, oracle_nets, oracle_lib):
    """A context over two device slots (both on GPU 0 here) shards gn_expand_and_evaluate by
    parents and gn_evaluate_games(with_children) by whole games (gn_partition) and returns
    exactly the single-device results."""
    from fishnet_amd import gpu_nnue as G
    one = G.GpuNnue(synth_big_path, synth_small_path, devices=[0])
    two = G.GpuNnue(synth_big_path, synth_small_path, devices=[0, 0])
    try:
        fens = special_fens() + random_fens(301, 31337)
        for mode in (0, 1):
            a, b = one.expand_and_evaluate(fens, mode), two.expand_and_evaluate(fens, mode)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), mode
        games = [("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1",
                  "e2e4 e7e5 g1f3 b8c6 f1b5 a7a6 b5a4 g8f6 e1g1 f8e7 f1e1 b7b5 a4b3 d7d6", (0, 3)),
                 ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", "e1g1 e8c8", ()),
                 ("4k3/8/8/8/8/8/4P3/4K3 w - - 0 1", "e2e4 e8d7 e4e5", (1,))] * 5
        ra, rb = one.evaluate_games(games, 0, children=True), two.evaluate_games(games, 0, children=True)
        for x, y in zip(ra, rb):
            assert x["status"] == y["status"] and np.array_equal(x["evals"], y["evals"])
            assert all(np.array_equal(c1[0], c2[0]) and np.array_equal(c1[1], c2[1])
                       for c1, c2 in zip(x["children"], y["children"]))
        big, small = oracle_nets
        fens0 = oracle_lib.replay_game(games[0][0], games[0][1])[0]
        for i, fen in enumerate(fens0):
            if i in (0, 3):
                continue
            p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, 0)
            assert tuple(rb[0]["evals"][i]) == p_exp
            mv, ev = rb[0]["children"][i]
            assert dict(zip(mv.tolist(), map(tuple, ev.tolist()))) == \
                dict(zip(m_exp, map(tuple, G.children_from_evals(k_exp).tolist())))
    finally:
        one.close()
        two.close()


def test_caller_stream_and_context_stream_do_not_race(gpu_ctx):
    """gn_evaluate_device on a caller stream returns while its kernels are queued; a call on
    the context stream right after must not overwrite the first call's library scratch
    (king-sort permutation, net outputs): each result equals its own synchronous run."""
    import ctypes
    from fishnet_amd import gpu_nnue as G
    n = 1 << 18
    bufs = [(gpu_ctx.alloc(n * 32), gpu_ctx.alloc(n * G.EVAL_SIZE)) for _ in range(2)]
    for k, (d_b, _) in enumerate(bufs):
        gpu_ctx.random_positions_device(100 + k, 0, n, 160, d_b)
    exp = []
    for d_b, d_o in bufs:
        gpu_ctx.evaluate_device(d_b, n, 0, d_o)
        gpu_ctx.synchronize()
        exp.append(d_o.download(G.EVAL_DTYPE, n))
    hip = ctypes.CDLL("libamdhip64.so")  # the runtime libgpu_nnue is linked against
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    try:
        for rep in range(3):
            for _, d_o in bufs:
                d_o.upload(np.zeros(n, dtype=G.EVAL_DTYPE))
            gpu_ctx.evaluate_device(bufs[0][0], n, 0, bufs[0][1], stream=s)
            gpu_ctx.evaluate_device(bufs[1][0], n, 0, bufs[1][1])
            gpu_ctx.synchronize()
            assert hip.hipStreamSynchronize(s) == 0
            for (_, d_o), e in zip(bufs, exp):
                assert np.array_equal(d_o.download(G.EVAL_DTYPE, n), e), rep
    finally:
        hip.hipStreamDestroy(s)


def test_common_row_base_under_int16_wrap_and_shared_kings(oracle_lib):
    """the common-row base with the int16-wrapping stress net, and tiles whose
    positions share their kings (and so the common rows) but differ in the side to move and
    the PSQT bucket: the per-position PSQT of the common rows at each position's own bucket."""
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(3072, 11, stress=True)
    ctx = G.GpuNnue(p, None)
    on = oracle_lib.Net(p)
    base = "r3k2r/pppq1ppp/2np1n2/2b1p3/2B1P3/2NP1N2/PPPQ1PPP/R3K2R {} KQkq - 0 1"
    fens = []
    # 16 positions: same kings and most pieces, stm alternating, pawns removed to change buckets
    pawns = ["a2", "b2", "c2", "f2", "g2", "h2", "a7", "b7"]
    for k in range(16):
        f = base.format("wb"[k & 1])
        board = oracle_lib._placement(f)
        for sq in pawns[:k // 2]:
            board.pop((int(sq[1]) - 1) * 8 + ord(sq[0]) - 97, None)
        rows = []
        for r in range(7, -1, -1):
            row, e = "", 0
            for fl in range(8):
                pc = board.get(r * 8 + fl)
                if pc is None:
                    e += 1
                else:
                    row += (str(e) if e else "") + pc
                    e = 0
            rows.append(row + (str(e) if e else ""))
        fens.append("/".join(rows) + " " + f.split(" ", 1)[1])
    fens = fens * 3 + special_fens() + random_fens(300, 4711)
    try:
        for ks in (2, 0):  # (2: sorted at any size; 1 sorts batches of >= 1,024)
            ctx.set_option(G.OPT_KING_SORT, ks)
            _cmp(ctx.evaluate_batch(fens, 1), oracle_lib.eval_fens(on, None, fens, 1, threads=8), fens)
    finally:
        ctx.close()


def test_nets_from_asset_archive(gpu_ctx, synth_big_path, synth_small_path, tmp_path):
    """gn_load_net_archive: both nets out of a zstd-compressed `ar` shaped like fishnet's
    assets.ar.zst (engine binary first, nets named nn-<sha256 prefix>.nnue), by name and
    by kind; results equal to the file-loaded context; a renamed (hash-mismatched)
    member is rejected."""
    import hashlib
    import archive_util as A
    from fishnet_amd import gpu_nnue as G
    big, small = open(synth_big_path, "rb").read(), open(synth_small_path, "rb").read()
    nb = "nn-" + hashlib.sha256(big).hexdigest()[:12] + ".nnue"
    ns = "nn-" + hashlib.sha256(small).hexdigest()[:12] + ".nnue"
    p = tmp_path / "assets.ar.zst"
    p.write_bytes(A.zstd(A.ar_bytes([("stockfish-x86-64-vnni512", b"\x7fELF" * 99), (nb, big), (ns, small)])))
    fens = special_fens() + random_fens(500, 0xA5C1)
    want = gpu_ctx.evaluate_batch(fens, 0)
    for kw in ({}, {"big_member": nb, "small_member": ns}):
        ctx = G.GpuNnue(archive=str(p), **kw)
        assert ctx.net_info() == gpu_ctx.net_info()
        assert np.array_equal(ctx.evaluate_batch(fens, 0), want)
        ctx.close()
    q = tmp_path / "renamed.ar.zst"
    q.write_bytes(A.zstd(A.ar_bytes([("nn-000000000000.nnue", big), (ns, small)])))
    with pytest.raises(G.GnError) as e:
        G.GpuNnue(archive=str(q), big_member="nn-000000000000.nnue")
    assert e.value.code == G.E_FORMAT


def _expand2(ctx, d_b, n, mode):
    """gn_expand2_device with buffers sized by its own E_CAPACITY replies."""
    from fishnet_amd import gpu_nnue as G
    out = {"po": ctx.alloc(n * G.EVAL_SIZE), "off": ctx.alloc((n + 1) * 4), "cap": 0, "gcap": 0}
    for _ in range(3):
        try:
            t, g = ctx.expand2_device(d_b, n, mode, out)
            return t, g, out
        except G.GnError as e:
            if e.code != G.E_CAPACITY:
                raise
            t, g = e.need
            if t > out["cap"]:
                out.update(cap=t, ch=ctx.alloc(max(t, 1) * 32), mv=ctx.alloc(max(t, 1) * 2),
                           co=ctx.alloc(max(t, 1) * G.EVAL_SIZE), goff=ctx.alloc((t + 1) * 4))
            if g > out["gcap"]:
                out.update(gcap=g, gmv=ctx.alloc(max(g, 1) * 2), gco=ctx.alloc(max(g, 1) * G.EVAL_SIZE))
    raise AssertionError("sizing did not converge")


@pytest.mark.parametrize("mode", [1, 0])
def test_grandchildren_vs_depth1_and_oracle(gpu_ctx, oracle_nets, oracle_lib, mode):
    """Depth 2 (gn_expand2_device): level 1 equals gn_expand_device; every grandchild
    equals a depth-1 expansion of its parent (the children as a parent batch, king cache
    off: refresh-started parents); sampled children's grandchildren equal the oracle's."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 3, 80
    n0 = games * (plies + 1)
    fens = special_fens()
    d_g = gpu_ctx.alloc(n0 * 32)
    gpu_ctx.random_games_device(0x5EED0077, 0, games, plies, d_g)
    gpu_ctx.synchronize()
    boards = np.concatenate([d_g.download(G.BOARD_DTYPE, n0), G.pack_fens(fens)[0]])
    n = len(boards)
    d_b = gpu_ctx.alloc(n * 32)
    d_b.upload(boards)
    t, g, out = _expand2(gpu_ctx, d_b, n, mode)
    assert t > 0 and g > 20 * t
    po, off = out["po"].download(G.EVAL_DTYPE, n), out["off"].download(np.uint32, n + 1)
    mv, co = out["mv"].download(np.uint16, t), out["co"].download(G.EVAL_DTYPE, t)
    goff = out["goff"].download(np.uint32, t + 1)
    gmv, gco = out["gmv"].download(np.uint16, g), out["gco"].download(G.EVAL_DTYPE, g)
    # level 1 == gn_expand_device
    b1 = {k: gpu_ctx.alloc(sz) for k, sz in (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("ch", t * 32), ("mv", t * 2),
                                              ("co", t * G.EVAL_SIZE))}
    assert gpu_ctx.expand_device(d_b, n, mode, b1["po"], b1["off"], b1["ch"], b1["mv"], b1["co"], t) == t
    assert np.array_equal(b1["po"].download(G.EVAL_DTYPE, n), po)
    assert np.array_equal(b1["co"].download(G.EVAL_DTYPE, t), co)
    # level 2 == depth 1 of the children with refresh-started parents (no chain, no cache)
    b2 = {k: gpu_ctx.alloc(sz) for k, sz in (("po", t * G.EVAL_SIZE), ("off", (t + 1) * 4), ("ch", g * 32), ("mv", g * 2),
                                              ("co", g * G.EVAL_SIZE))}
    try:
        gpu_ctx.set_option(G.OPT_CHAIN, 1)
        gpu_ctx.set_option(G.OPT_KING_CACHE, 0)
        assert gpu_ctx.expand_device(out["ch"], t, mode, b2["po"], b2["off"], b2["ch"], b2["mv"], b2["co"], g) == g
    finally:
        gpu_ctx.set_option(G.OPT_CHAIN, 81)
        gpu_ctx.set_option(G.OPT_KING_CACHE, 1)
    assert static_part(b2["po"].download(G.EVAL_DTYPE, t)) == static_part(co)  # scored positions vs child records
    assert np.array_equal(b2["off"].download(np.uint32, t + 1), goff)
    assert np.array_equal(b2["mv"].download(np.uint16, g), gmv)
    assert np.array_equal(b2["co"].download(G.EVAL_DTYPE, g), gco)
    # sampled children against the oracle
    big, small = oracle_nets
    children = out["ch"].download(G.BOARD_DTYPE, t)
    rng = np.random.default_rng(7)
    for j in np.unique(np.concatenate([rng.choice(t, size=min(200, t), replace=False), np.arange(40)])):
        fen = G.board_to_fen(children[j])
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, mode)
        assert static_part(co[j:j + 1]) == static_part(np.array([p_exp], dtype=G.EVAL_DTYPE)), fen
        assert co[j]["flags"] & G.FLAG_NO_SCORE
        lo, hi = int(goff[j]), int(goff[j + 1])
        assert {int(m): tuple(x) for m, x in zip(gmv[lo:hi], gco[lo:hi])} == \
               {int(m): tuple(x) for m, x in zip(m_exp, k_exp)}, fen



def _expand_runner(ctx, d_b, n, cap, mode=1):
    """expand_device with the given chain / king-cache options into fresh buffers."""
    from fishnet_amd import gpu_nnue as G
    bufs = {k: ctx.alloc(sz) for k, sz in (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("ch", cap * 32),
                                              ("mv", cap * 2), ("co", cap * G.EVAL_SIZE))}

    def run(k, kc, inc=1):
        ctx.set_option(G.OPT_CHAIN, k)
        ctx.set_option(G.OPT_KING_CACHE, kc)
        ctx.set_option(G.OPT_INCREMENTAL_CHILDREN, inc)
        try:
            t = ctx.expand_device(d_b, n, mode, bufs["po"], bufs["off"], bufs["ch"], bufs["mv"], bufs["co"], cap)
        finally:
            ctx.set_option(G.OPT_CHAIN, 81)
            ctx.set_option(G.OPT_KING_CACHE, 1)
            ctx.set_option(G.OPT_INCREMENTAL_CHILDREN, 1)
        return (bufs["po"].download(G.EVAL_DTYPE, n), bufs["off"].download(np.uint32, n + 1),
                bufs["mv"].download(np.uint16, t), bufs["co"].download(G.EVAL_DTYPE, t))
    return run


def _check_vs_oracle(oracle_lib, big, fens, res, mode=1):
    parents, offs, moves, kids = res
    for i, fen in enumerate(fens):
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, None, fen, mode)
        assert tuple(parents[i]) == p_exp, fen
        lo, hi = int(offs[i]), int(offs[i + 1])
        assert {int(m): tuple(x) for m, x in zip(moves[lo:hi], kids[lo:hi])} == \
               {int(m): tuple(x) for m, x in zip(m_exp, k_exp)}, fen


@pytest.mark.parametrize("stress", [False, True])
def test_l1_1024_planned_expansion(oracle_lib, stress):
    """the planned path is the default for L1 = 1024 nets too (plan_kernel<1024> +
    stream_eval_kernel<1024>: 2 waves of 128 threads, the rotating finishing wave, 8 k-steps per
    wave, 2,176-B rows).  Chained walk and king cache on and off and the full-refresh path give
    identical results, and the first games equal the oracle, on a normal and an int16-wrap net."""
    from fishnet_amd import gpu_nnue as G, synthnet
    p = synthnet.cached_synth_net(1024, 5, stress=stress)
    ctx = G.GpuNnue(p, None)
    try:
        assert ctx.net_info()["big_l1"] == 1024
        games, plies = 30, 80
        n = games * (plies + 1)
        d_b = ctx.alloc(n * 32)
        ctx.random_games_device(0x5EED1024, 0, games, plies, d_b)
        ctx.synchronize()
        run = _expand_runner(ctx, d_b, n, 60 * n)
        ref = run(1, 0, inc=0)  # every position a full refresh (eval_net<1024>)
        for k, kc in ((1, 0), (-81, 1), (-81, 0), (-5, 1), (81, 1)):
            got = run(k, kc)
            assert all(np.array_equal(a, b) for a, b in zip(ref, got)), (k, kc)
        on = oracle_lib.Net(p)
        fens = [G.board_to_fen(b) for b in d_b.download(G.BOARD_DTYPE, 2 * (plies + 1))]
        _check_vs_oracle(oracle_lib, on, fens, ref)
    finally:
        ctx.close()


def test_king_cache_reload_at_minimum_gap(gpu_ctx, oracle_nets, oracle_lib):
    """a king-cache row reloaded right after its store.  Kings shuffling
    e1-e2 / e8-e7 make every parent and every king-move child hit the rows the previous
    positions stored; the plan pads each such reload to exactly GN_SCR_GAP list entries behind
    the store (GN_STAT_SCRATCH_PADS > 0: the minimum distance occurred), the plan's error word
    (bit 2: a reload closer than that; checked after every planned expansion) stays clear, and
    the results equal the refresh path and the oracle."""
    from fishnet_amd import gpu_nnue as G
    shuffle = "e2e4 e7e5 " + " ".join(["e1e2 e8e7 e2e1 e7e8"] * 19) + " e1e2 e8e7"
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    fens, _ = oracle_lib.replay_game(start, shuffle)
    assert len(fens) == 81
    boards = np.tile(G.pack_fens(fens)[0], 24)
    n = len(boards)
    d_b = gpu_ctx.alloc(n * 32)
    d_b.upload(boards)
    run = _expand_runner(gpu_ctx, d_b, n, 40 * n)
    ref = run(1, 0)
    got = run(-81, 1)
    pads = gpu_ctx.get_option(G.STAT_SCRATCH_PADS)
    assert pads > 0
    assert all(np.array_equal(a, b) for a, b in zip(ref, got))
    big, _ = oracle_nets
    _check_vs_oracle(oracle_lib, big, fens, tuple(x[:81] if i == 0 else x for i, x in enumerate(got)))


def test_pipeline_chunks_equal_one_chunk(gpu_ctx):
    """The host-buffer expansion pipeline cut into many chunks (GN_OPT_CHUNK_PARENTS: slot reuse in
    the device output buffers, the drain threads' downloads on the copy stream, chunk cuts at game
    starts) returns byte-identical results to one chunk: gn_evaluate_games with children (cuts at
    game starts, skipped positions inside chunks) and gn_expand_and_evaluate (cuts every 81), with
    the chunks overlapped (GN_OPT_EXPAND_PIPELINE 1: chunk c + 1's children and plan on the second
    stream while chunk c finishes; 2, the default: beside chunk c's row stream) and one after
    another."""
    from fishnet_amd import gpu_nnue as G
    ucis = G.random_games_uci(0x5EED0123, 0, 40, 80)
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    games = [(start, u, (3, 17) if g % 3 == 0 else ()) for g, u in enumerate(ucis)]
    arr, keep = G._games_array(games)
    fens = [G.board_to_fen(b) for b in G.random_positions(0x5EED0456, 0, 700, 160)]
    try:
        out = {}
        for chunk, pipe in ((0, 2), (100, 1), (250, 1), (100, 0), (250, 0), (100, 2), (250, 2)):
            gpu_ctx.set_option(G.OPT_CHUNK_PARENTS, chunk)
            gpu_ctx.set_option(G.OPT_EXPAND_PIPELINE, pipe)
            res = gpu_ctx.evaluate_games_arrays(arr, len(games), 0, children=True)
            out[chunk, pipe] = ([np.copy(x) for x in res[:6]], [np.copy(x) for x in gpu_ctx.expand_and_evaluate(fens, 1)])
        for key in ((100, 1), (250, 1), (100, 0), (250, 0), (100, 2), (250, 2)):
            for a, b in zip(out[0, 2][0] + out[0, 2][1], out[key][0] + out[key][1]):
                assert a.tobytes() == b.tobytes(), key
    finally:
        gpu_ctx.set_option(G.OPT_CHUNK_PARENTS, 0)
        gpu_ctx.set_option(G.OPT_EXPAND_PIPELINE, 2)


def test_concurrent_batches_coalesce(gpu_ctx):
    """16 threads calling gn_evaluate_batch at once on one context (fishnet's workers, one
    chunk each): the calls are merged into shared launches (GN_OPT_COALESCE) and every caller
    gets exactly the records of a call on its own, with coalescing on and off; the threads use all
    three modes (merged launches of different modes run at once, two per class in flight)."""
    import threading
    from fishnet_amd import gpu_nnue as G
    lists = [[G.board_to_fen(b) for b in G.random_positions(0x5EED0900 + t, 0, 81, 160)] for t in range(16)]
    lists[3][5] = "not a fen"  # a bad FEN is flagged in its own call only
    ref = [gpu_ctx.evaluate_batch(fl, t % 3) for t, fl in enumerate(lists)]
    assert ref[3][5]["flags"] & G.FLAG_BAD_FEN
    for coalesce in (1, 0):
        gpu_ctx.set_option(G.OPT_COALESCE, coalesce)
        l0, c0 = gpu_ctx.get_option(G.STAT_BATCH_LAUNCHES), gpu_ctx.get_option(G.STAT_BATCH_CALLS)
        got, errs = [None] * 16, []
        go = threading.Barrier(16)

        def work(t):
            try:
                go.wait()
                for _ in range(4):
                    got[t] = gpu_ctx.evaluate_batch(lists[t], t % 3)
            except Exception as e:  # surfaced below
                errs.append(e)

        th = [threading.Thread(target=work, args=(t,)) for t in range(16)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs
        for t in range(16):
            assert np.array_equal(got[t], ref[t]), (coalesce, t)
        launches = gpu_ctx.get_option(G.STAT_BATCH_LAUNCHES) - l0
        calls = gpu_ctx.get_option(G.STAT_BATCH_CALLS) - c0
        if coalesce:
            assert calls == 64 and 1 <= launches < calls, (launches, calls)
        else:
            assert calls == 0 and launches == 0
    gpu_ctx.set_option(G.OPT_COALESCE, 1)


def test_eval_params_keep_child_cp_in_24_bits(gpu_ctx):
    """gn_child holds final_cp in 24 bits: gn_set_eval_params refuses a win-rate model whose
    a(material) drops below 1 anywhere in the clamped material range (|final_cp| then stays
    <= 100 * value_clamp < 2^23), and accepts the defaults back."""
    from fishnet_amd import gpu_nnue as G
    p = gpu_ctx.eval_params()
    bad = gpu_ctx.eval_params()
    bad.wdl_a[3] = 0.5 - (bad.wdl_a[0] + bad.wdl_a[1] + bad.wdl_a[2])  # a(1.0) = 0.5
    bad.wdl_material_anchor = 58
    bad.wdl_material_min, bad.wdl_material_max = 58, 58
    with pytest.raises(G.GnError) as e:
        gpu_ctx.set_eval_params(bad)
    assert e.value.code == G.E_INVALID
    gpu_ctx.set_eval_params(p)
    assert gpu_ctx.eval_params().wdl_a[3] == p.wdl_a[3]


@pytest.mark.gpu
def test_stream_column_slices_equal_whole_rows(gpu_ctx, oracle_nets, oracle_lib):
    """GN_OPT_STREAM_SLICES: the big net's stream as three launches over 1,024 accumulator
    columns each (every slice stores its fc_0 partial sums; finalize adds the three where it reads
    each big-net output and runs the rest of the layer stack, slice_finish_one -- the separate
    slice_finish_kernel runs only in the -DGN_AB_FINISH_SEPARATE A/B build) gives every output of the one-launch whole-row stream, with
    the chained walk and king cache on and off, in mode BIG (every position on the big net) and
    mode FULL (the big net on the positions the small net hands over: gaps in the slices' position
    lists); sampled parents with all their children against the oracle."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 1200, 80
    n = games * (plies + 1)
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0000 + 1200, 0, games, plies, d_b)
    gpu_ctx.synchronize()
    _, total, _, _ = gpu_ctx.time_expand_device(d_b, n, 1, 1)
    out = {"po": gpu_ctx.alloc(n * G.EVAL_SIZE), "off": gpu_ctx.alloc((n + 1) * 4), "mv": gpu_ctx.alloc(total * 2),
           "co": gpu_ctx.alloc(total * G.EVAL_SIZE), "cap": total}

    def run(slices, k, kc, mode=1):
        gpu_ctx.set_option(G.OPT_STREAM_SLICES, slices)
        gpu_ctx.set_option(G.OPT_CHAIN, k)
        gpu_ctx.set_option(G.OPT_KING_CACHE, kc)
        _, t, _, _ = gpu_ctx.time_expand_device(d_b, n, mode, 1, outputs=out)
        assert t == total
        return tuple(gpu_ctx.checksum_device(out[b], nb) for b, nb in
                     (("po", n * G.EVAL_SIZE), ("co", t * G.EVAL_SIZE)))

    assert gpu_ctx.get_option(G.OPT_STREAM_SLICES) == 3
    try:
        for k, kc, mode in ((81, 1, 1), (1, 0, 1), (81, 1, 0), (1, 0, 0)):
            whole = run(1, k, kc, mode)
            assert run(3, k, kc, mode) == whole, (k, kc, mode)
        with pytest.raises(G.GnError):
            gpu_ctx.set_option(G.OPT_STREAM_SLICES, 2)
    finally:
        gpu_ctx.set_option(G.OPT_STREAM_SLICES, 3)
        gpu_ctx.set_option(G.OPT_CHAIN, 81)
        gpu_ctx.set_option(G.OPT_KING_CACHE, 1)
    run(3, 81, 1)
    big, small = oracle_nets
    boards = d_b.download(G.BOARD_DTYPE, n)
    offs = out["off"].download(np.uint32, n + 1)
    pev = out["po"].download(G.EVAL_DTYPE, n)
    rng = np.random.default_rng(3)
    for i in rng.choice(n, 48, replace=False):
        fen = G.board_to_fen(boards[i])
        lo, hi = int(offs[i]), int(offs[i + 1])
        mv = out["mv"].download(np.uint16, hi - lo, offset=lo)
        ev = out["co"].download(G.EVAL_DTYPE, hi - lo, offset=lo)
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, 1, incremental=True)
        assert tuple(pev[i]) == p_exp, fen
        assert dict(zip(mv.tolist(), map(tuple, ev.tolist()))) == dict(zip(m_exp, map(tuple, k_exp.tolist()))), fen


_FAULT_CHILD = r"""
import json, sys
import numpy as np
from fishnet_amd import gpu_nnue as G
big, small, games = sys.argv[1], sys.argv[2], int(sys.argv[3])
ctx = G.GpuNnue(big, small, devices=[0])
n = games * 81
d_b = ctx.alloc(n * 32)
ctx.random_games_device(0x5EED0FA1, 0, games, 80, d_b)
ctx.synchronize()
ctx.set_option(G.OPT_CHAIN, -81)  # one block per game: block 1 exists
res = {}
try:
    ctx.time_expand_device(d_b, n, G.MODE_BIG, 1)
    res["first"] = "ok"
except G.GnError as e:
    res["first"] = [e.code, str(e)]
_, total, _, _ = ctx.time_expand_device(d_b, n, G.MODE_BIG, 1)
out = {"po": ctx.alloc(n * G.EVAL_SIZE), "off": ctx.alloc((n + 1) * 4), "mv": ctx.alloc(total * 2),
       "co": ctx.alloc(total * G.EVAL_SIZE), "cap": total}
_, t, _, _ = ctx.time_expand_device(d_b, n, G.MODE_BIG, 1, outputs=out)
res["second"] = [ctx.checksum_device(out[b], nb) for b, nb in
                 (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("mv", t * 2), ("co", t * G.EVAL_SIZE))]
ctx.close()
print(json.dumps(res), flush=True)
"""


def test_plan_overflow_fails_the_call_then_recovers(gpu_ctx, synth_big_path, synth_small_path):
    """round 4's plan bug made the plan overflow its lists; the plan reported it
    (err bit 0) but the stream, launched before the host reads the error word, followed the bad
    tile ends and faulted.  The stream now clamps every tile end to the block's entry region.
    The fault-injection build (fishnet_amd/build.py FAULT_LIB, -DGN_FAULT_PLAN_BLOCK=1) has the
    plan report an overflow for block 1 on its first launch and leave that block's last tile ends
    4,096 entries past the region: in a process of its own (the variant library), the expansion
    returns GN_E_HIP naming error bit 0 -- no fault -- and the next expansion on the same context
    returns exactly the normal library's records (device checksums of every output)."""
    import subprocess
    import sys
    from fishnet_amd import build, gpu_nnue as G
    assert os.path.exists(build.FAULT_LIB), "run __graft_entry__.build() (builds the fault-injection library)"
    games = 6
    env = dict(os.environ, GPU_NNUE_LIB=build.FAULT_LIB)
    p = subprocess.run([sys.executable, "-c", _FAULT_CHILD, synth_big_path, synth_small_path, str(games)],
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["first"][0] == G.E_HIP and "0x1" in res["first"][1], res["first"]
    # the same expansion with the normal library, in this process
    n = games * 81
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0FA1, 0, games, 80, d_b)
    gpu_ctx.synchronize()
    try:
        gpu_ctx.set_option(G.OPT_CHAIN, -81)
        _, total, _, _ = gpu_ctx.time_expand_device(d_b, n, G.MODE_BIG, 1)
        out = {"po": gpu_ctx.alloc(n * G.EVAL_SIZE), "off": gpu_ctx.alloc((n + 1) * 4), "mv": gpu_ctx.alloc(total * 2),
               "co": gpu_ctx.alloc(total * G.EVAL_SIZE), "cap": total}
        _, t, _, _ = gpu_ctx.time_expand_device(d_b, n, G.MODE_BIG, 1, outputs=out)
    finally:
        gpu_ctx.set_option(G.OPT_CHAIN, 81)
    exp = [gpu_ctx.checksum_device(out[b], nb) for b, nb in
           (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("mv", t * 2), ("co", t * G.EVAL_SIZE))]
    assert res["second"] == exp


def test_two_device_slots_games_at_scale(synth_big_path, synth_small_path, oracle_nets, oracle_lib):
    """the in-process multi-device path (one host thread per device slot,
    INTEGRATION.md section 5) at the bench's shape -- 1,024 lichess-shaped 80-ply games through
    gn_evaluate_games(with_children) with the column-sliced stream on two device slots (both on
    GPU 0 here: gn_partition gives each slot 512 whole games, each runs its own chained walk,
    king cache and three slice launches) -- returns byte for byte the single-slot records, and
    sampled positions with all their children equal the oracle."""
    from fishnet_amd import gpu_nnue as G
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    games = [(start, u, (5,) if g % 7 == 0 else ()) for g, u in enumerate(G.random_games_uci(0x5EED2D2D, 0, 1024, 80))]
    arr, keep = G._games_array(games)
    res = []
    for devs in ([0], [0, 0]):
        ctx = G.GpuNnue(synth_big_path, synth_small_path, devices=devs)
        try:
            assert ctx.get_option(G.OPT_STREAM_SLICES) == 3
            res.append([np.copy(x) for x in ctx.evaluate_games_arrays(arr, len(games), G.MODE_BIG, children=True)[:6]])
        finally:
            ctx.close()
    for a, b in zip(*res):
        assert a.tobytes() == b.tobytes()
    offs, status, pos, coffs, cmoves, kids = res[1]
    npos = int(offs[-1])  # (a random game may end early, at mate or a draw)
    assert not status.any() and npos > 1024 * 70 and int(coffs[npos]) > npos * 20
    big, _ = oracle_nets
    rng = np.random.default_rng(11)
    for g in rng.choice(len(games), 4, replace=False):
        fens = oracle_lib.replay_game(start, games[g][1])[0]
        ng = int(offs[g + 1] - offs[g])
        assert ng == len(fens)
        for i in (0, ng // 2, ng - 1):
            k = int(offs[g]) + i
            p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, None, fens[i], G.MODE_BIG)
            assert tuple(pos[k]) == p_exp, (g, i)
            lo, hi = int(coffs[k]), int(coffs[k + 1])
            got = dict(zip(cmoves[lo:hi].tolist(), map(tuple, G.decode_children(kids[lo:hi]).tolist())))
            assert got == dict(zip(m_exp, map(tuple, G.children_from_evals(k_exp).tolist()))), (g, i)


def test_fast_batch_graph_equals_general_path(gpu_ctx, oracle_nets, oracle_lib):
    """The drop-in's small-batch graphs (GN_OPT_FAST_BATCH, gpu_nnue.hip FastBatch): one lichess
    game per call as GpuEvalStub sends it, batches at the size-class edges, every mode, a batch
    whose in-check replies overflow the graph's capacity (rerun on the general path), one whose
    in-check positions are packed together (reply_level_kernel's per-thread overflow), and new
    eval params (the graphs are recaptured) -- every record equal to the general path's, and a
    sample of games against the oracle."""
    from fishnet_amd import gpu_nnue as G
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"
    games = [G.boards_to_fens(G.replay_game(start, u)[0]) for u in G.random_games_uci(0x5EED0A00, 0, 24, 80)]
    big, small = oracle_nets
    # (positions of random games: ~4 % are in check; gn_random_positions gave none of 4,200 in
    # check, the oracle agrees)
    pool = [f for u in G.random_games_uci(0x5EED0A01, 0, 60, 80) for f in G.boards_to_fens(G.replay_game(start, u)[0])]
    pool = pool[:4200] + special_fens()
    fl = gpu_ctx.evaluate_batch(pool, 1)["flags"]
    checks = [f for f, x in zip(pool, fl) if x & G.FLAG_IN_CHECK and not x & G.FLAG_NO_MOVES]
    assert len(checks) >= 50
    quiet = [f for f, x in zip(pool, fl) if not x & G.FLAG_IN_CHECK]
    # in-check positions packed together: reply_level_kernel's threads hold 16 positions each at
    # 4,096, so the first threads' replies overflow their LDS segments (written by the thread itself)
    dense = (checks * 2)[:60] + quiet[:4096 - 60]
    batches = games + [pool[:1], pool[:127], pool[:128], pool[:129], pool[:1000], pool[:4096], dense, pool[:4097]]
    overflow = (checks * 40)[:1000]  # 1,000 in-check positions: their replies exceed 1024 / 2 + 256

    def run(fens, mode, fast):
        gpu_ctx.set_option(G.OPT_FAST_BATCH, fast)
        return gpu_ctx.evaluate_batch(fens, mode)

    try:
        for mode in (0, 1, 2):
            f0, fb0 = gpu_ctx.get_option(G.STAT_FAST_BATCHES), gpu_ctx.get_option(G.STAT_FAST_FALLBACKS)
            for fens in batches + [overflow]:
                assert np.array_equal(run(fens, mode, 1), run(fens, mode, 0)), (mode, len(fens))
            # every batch but the 4,097 ran a graph, and the overflowing one fell back
            assert gpu_ctx.get_option(G.STAT_FAST_BATCHES) - f0 == len(batches) - 1 + 1
            assert gpu_ctx.get_option(G.STAT_FAST_FALLBACKS) - fb0 == 1
            for fens in games[:4]:
                _cmp(run(fens, mode, 1), oracle_lib.eval_fens(big, small, fens, mode), fens)
        p = gpu_ctx.eval_params()
        q = gpu_ctx.eval_params()
        q.psqt_weight, q.rule50_div = 111, 150
        gpu_ctx.set_eval_params(q)
        for fens in games[:3] + [pool[:300]]:
            assert np.array_equal(run(fens, 0, 1), run(fens, 0, 0))
        gpu_ctx.set_eval_params(p)
        assert np.array_equal(run(games[0], 0, 1), run(games[0], 0, 0))
    finally:
        gpu_ctx.set_option(G.OPT_FAST_BATCH, 1)


_ODD_CHILD = r"""
import sys
import numpy as np
from fishnet_amd import gpu_nnue as G
big, small, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
fens = [G.board_to_fen(b) for b in G.random_positions(0x5EED0DD5, 0, n, 160)]
ctx = G.GpuNnue(big, small, devices=[0])
np.save(out, np.stack([ctx.evaluate_batch(fens, m) for m in (G.MODE_SMALL, G.MODE_FULL)]))
ctx.close()
"""


def test_small_net_odd_gather_depth_vs_oracle(gpu_ctx, synth_big_path, synth_small_path, oracle_nets, oracle_lib,
                                              tmp_path):
    """eval_net<128>'s gather keeps GN_SMALL_DEPTH rows in flight (default 4); an odd
    depth adds its last row on its own and takes a tail of up to D - 1 rows.  The variant library
    built with depth 5 (fishnet_amd/build.py ODD_LIB), in a process of its own, evaluates 4,096
    random-playout positions (2..32 pieces: every remainder of the row count mod 5) in modes SMALL
    and FULL: equal to the oracle and to the default library."""
    import subprocess
    import sys
    from fishnet_amd import build, gpu_nnue as G
    assert os.path.exists(build.ODD_LIB), "run __graft_entry__.build() (builds the odd-depth library)"
    n = 4096
    dst = str(tmp_path / "odd.npy")
    env = dict(os.environ, GPU_NNUE_LIB=build.ODD_LIB)
    p = subprocess.run([sys.executable, "-c", _ODD_CHILD, synth_big_path, synth_small_path, str(n), dst],
                       env=env, cwd=os.path.dirname(HERE), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    got = np.load(dst)
    fens = [G.board_to_fen(b) for b in G.random_positions(0x5EED0DD5, 0, n, 160)]
    big, small = oracle_nets
    for k, m in enumerate((G.MODE_SMALL, G.MODE_FULL)):
        assert np.array_equal(got[k], gpu_ctx.evaluate_batch(fens, m)), m
        assert np.array_equal(got[k], oracle_lib.eval_fens(big, small, fens, m)), m


def test_expand_pipeline_equals_serial(gpu_ctx, oracle_nets, oracle_lib):
    """GN_OPT_EXPAND_PIPELINE: gn_time_expand_device's iterations overlapped (expansion k + 1's
    children and plan on the second stream, in the other buffer set, while expansion k's finalize
    and score rule run) give every output of one serial expansion -- parents, offsets, moves,
    children -- in modes BIG and FULL, for 2 and 3 iterations (each buffer set used as the last);
    sampled parents with all their children against the oracle."""
    from fishnet_amd import gpu_nnue as G
    games, plies = 300, 80
    n = games * (plies + 1)
    d_b = gpu_ctx.alloc(n * 32)
    gpu_ctx.random_games_device(0x5EED0F1F, 0, games, plies, d_b)
    gpu_ctx.synchronize()
    _, total, _, _ = gpu_ctx.time_expand_device(d_b, n, 1, 1)
    out = {"po": gpu_ctx.alloc(n * G.EVAL_SIZE), "off": gpu_ctx.alloc((n + 1) * 4), "mv": gpu_ctx.alloc(total * 2),
           "co": gpu_ctx.alloc(total * G.EVAL_SIZE), "cap": total}

    def run(iters, pipe, mode):
        gpu_ctx.set_option(G.OPT_EXPAND_PIPELINE, pipe)
        for b in ("po", "off", "mv", "co"):
            out[b].upload(np.zeros(out[b].nbytes, np.uint8))
        _, t, _, _ = gpu_ctx.time_expand_device(d_b, n, mode, iters, outputs=out)
        assert t == total
        return tuple(gpu_ctx.checksum_device(out[b], nb) for b, nb in
                     (("po", n * G.EVAL_SIZE), ("off", (n + 1) * 4), ("mv", t * 2), ("co", t * G.EVAL_SIZE)))

    assert gpu_ctx.get_option(G.OPT_EXPAND_PIPELINE) == 2
    try:
        for mode in (1, 0):
            serial = run(1, 0, mode)
            for pipe in (1, 2):  # (2: the next front beside the row stream)
                assert run(2, pipe, mode) == serial, (mode, pipe)
                assert run(3, pipe, mode) == serial, (mode, pipe)
            assert run(3, 0, mode) == serial, mode
    finally:
        gpu_ctx.set_option(G.OPT_EXPAND_PIPELINE, 2)
    run(3, 2, 1)  # pipelined, mode BIG: sampled parents with all their children against the oracle
    big, small = oracle_nets
    parents = d_b.download(G.BOARD_DTYPE, n)
    offs = out["off"].download(np.uint32, n + 1)
    pev = out["po"].download(G.EVAL_DTYPE, n)
    for i in np.random.default_rng(5).choice(n, 24, replace=False):
        lo, hi = int(offs[i]), int(offs[i + 1])
        mv = out["mv"].download(np.uint16, hi - lo, offset=lo)
        ev = out["co"].download(G.EVAL_DTYPE, hi - lo, offset=lo)
        p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, G.board_to_fen(parents[i]), 1, incremental=True)
        assert tuple(pev[i]) == p_exp
        assert dict(zip(mv.tolist(), map(tuple, ev.tolist()))) == dict(zip(m_exp, map(tuple, k_exp.tolist())))
