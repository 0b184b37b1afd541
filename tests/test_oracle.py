"""The CPU oracle pinned before it is trusted (CPU only).

- movegen: public perft known answers (tests/golden/perft.json), incl. Chess960;
- NNUE: "parity unpinned" against Stockfish (no source, binary or net exists in
  the container).  What IS pinned: the committed goldens
  (regression), hand-derived HalfKAv2_hm indices, the file format round trip,
  and a third, independent numpy restatement written here in the test.
"""
import hashlib
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def test_perft_known_answers(oracle_lib):
    g = json.load(open(os.path.join(HERE, "golden", "perft.json")))
    for c in g["cases"]:
        for d, nodes in enumerate(c["nodes"], start=1):
            if nodes > 3_000_000:
                break
            assert oracle_lib.perft(c["fen"], d) == nodes, (c["name"], d)


def test_hashes_two_implementations(oracle_lib):
    from fishnet_amd import synthnet
    for l1 in (128, 1024, 3072):
        assert oracle_lib.expected_hash(l1) == synthnet.hashes(l1)


def test_leb128_roundtrip():
    from fishnet_amd import synthnet
    rng = np.random.default_rng(0)
    for bits in (16, 32):
        lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
        v = np.concatenate([np.array([0, 1, -1, 63, 64, -64, -65, lo, hi]),
                            rng.integers(lo, hi, 2000)]).astype(np.int64)
        assert np.array_equal(synthnet.leb128_decode(synthnet.leb128_encode(v), len(v), bits), v)


def test_feature_index_hand_derived(oracle_lib):
    # white perspective, white king e1 (file e: no mirror, bucket 31 -> 21824)
    w = oracle_lib.features(START, 0)
    assert 8 + 21824 in w          # own pawn a2: plane 0
    assert 60 + 640 + 21824 in w   # their king e8: plane 10
    assert 57 + 3 * 64 + 21824 in w  # their knight b8: plane 3
    # black perspective is the mirror image of white's at the start position
    assert sorted(oracle_lib.features(START, 1)) == sorted(w)
    # king on d1 (file d) mirrors files: own rook a1 -> a1 ^ 7 = h1 (7), bucket 28+3=31
    f = oracle_lib.features("4k3/8/8/8/8/8/8/R2K4 w - - 0 1", 0)
    assert 7 + 6 * 64 + 31 * 704 in f
    # white king on h1: file h (no mirror), bucket 4*7 + min(7, 0) = 28
    f = oracle_lib.features("k7/8/8/8/8/8/8/7K w - - 0 1", 0)
    assert 7 + 640 + 28 * 704 in f and 56 + 640 + 28 * 704 in f
    # black perspective, black king a8: files a-d mirror, ranks flip -> a8 ^ 63 = h1, bucket 28
    f = oracle_lib.features("k7/8/8/8/8/8/8/7K w - - 0 1", 1)
    assert (56 ^ 63) + 640 + 28 * 704 in f and (7 ^ 63) + 640 + 28 * 704 in f
    assert all(0 <= x < 22528 for x in f)


def test_goldens_regenerate_identically(oracle_lib, oracle_nets, synth_big_path, synth_small_path):
    g = json.load(open(os.path.join(HERE, "golden", "eval_goldens.json")))
    sha = lambda p: hashlib.sha256(open(p, "rb").read()).hexdigest()
    assert g["nets"]["big"]["sha256"] == sha(synth_big_path)
    assert g["nets"]["small"]["sha256"] == sha(synth_small_path)
    big, small = oracle_nets
    for name, mode in (("full", 0), ("big", 1), ("small", 2)):
        rows = g["results"][name]
        got = oracle_lib.eval_fens(big, small, [r[0] for r in rows], mode, threads=4)
        assert [list(map(int, r)) for r in got.tolist()] == [r[1:] for r in rows]


def test_goldens_cover_every_branch():
    g = json.load(open(os.path.join(HERE, "golden", "eval_goldens.json")))
    fi = g["columns"].index("flags")
    flags = [r[fi] for r in g["results"]["full"]]
    assert any(f & 1 for f in flags) and any(f & 2 for f in flags) and any(f & 8 for f in flags)
    assert any(f & 10 == 0 for f in flags)


def py_to_cp(v, fen):
    """Third restatement of UCIEngine::to_cp (win_rate_params' a(material)), Python floats
    (IEEE double, no contraction) with std::round's half-away-from-zero."""
    w = {"p": 1, "n": 3, "b": 3, "r": 5, "q": 9}
    material = sum(w.get(ch.lower(), 0) for ch in fen.split()[0] if ch.isalpha())
    m = min(max(material, 17), 78) / 58.0
    a = (((-37.45051876 * m + 121.19101539) * m + -132.78783573) * m) + 420.70576692
    x = 100 * v / a
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


def test_final_cp_restated_three_ways(oracle_lib, oracle_nets):
    """final_cp of every golden row = to_cp(final_v) by an independent Python restatement, and
    hand-computed anchors: a(58 material) = sum of the coefficients = 371.1484..."""
    g = json.load(open(os.path.join(HERE, "golden", "eval_goldens.json")))
    ci, vi = g["columns"].index("final_cp"), g["columns"].index("final_v")
    n = 0
    for rows in g["results"].values():
        for r in rows:
            assert r[ci] == py_to_cp(r[vi], r[0]), r
            n += 1
    assert n > 200
    start = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"  # material 78 (clamped at 78)
    assert py_to_cp(372, "4k3/8/8/8/8/8/8/4K3 w - - 0 1") == round(37200 / (((-37.45051876 * (17 / 58) + 121.19101539)
                                                                            * (17 / 58) - 132.78783573) * (17 / 58) + 420.70576692))
    m = 78 / 58.0
    a78 = ((-37.45051876 * m + 121.19101539) * m - 132.78783573) * m + 420.70576692
    assert py_to_cp(-1000, start) == -round(100000 / a78)


# ---------------------------------------------------------------- numpy ----
PT = {"p": 1, "n": 2, "b": 3, "r": 4, "q": 5, "k": 6}


def np_board(fen):
    rows, stm = fen.split()[0].split("/"), fen.split()[1]
    pcs = {}
    for r, row in enumerate(rows):
        f = 0
        for ch in row:
            if ch.isdigit():
                f += int(ch)
            else:
                pcs[(7 - r) * 8 + f] = (0 if ch.isupper() else 1, PT[ch.lower()])
                f += 1
    rule50 = int(fen.split()[4]) if len(fen.split()) > 4 else 0
    return pcs, (1 if stm == "b" else 0), rule50


def np_index(persp, sq, color, pt, ksq):
    kf = ksq % 8
    orient = (7 if kf < 4 else 0) ^ (56 if persp else 0)
    rr = (ksq // 8) ^ (7 if persp else 0)
    bucket = 4 * (7 - rr) + min(kf, 7 - kf)
    plane = 10 if pt == 6 else 2 * (pt - 1) + (color != persp)
    return (sq ^ orient) + 64 * plane + 704 * bucket


def np_net_output(a, fen):
    """numpy restatement of Network::evaluate for a synthetic net's arrays."""
    pcs, stm, _ = np_board(fen)
    l1 = a["ft_bias"].shape[0]
    h = l1 // 2
    acc, ps = {}, {}
    for persp in (0, 1):
        ksq = [s for s, (c, t) in pcs.items() if c == persp and t == 6][0]
        idx = [np_index(persp, s, c, t, ksq) for s, (c, t) in pcs.items()]
        w = a["ft_w"][idx].astype(np.int64).sum(axis=0) * 2 + a["ft_bias"].astype(np.int64) * 2
        acc[persp] = ((w + 32768) % 65536 - 32768)  # int16 wrap of the doubled sum
        ps[persp] = a["psqt"][idx].astype(np.int64).sum(axis=0)
    x = np.concatenate([np.clip(acc[p][:h], 0, 254) * np.clip(acc[p][h:], 0, 254) // 512 for p in (stm, 1 - stm)])
    bucket = (len(pcs) - 1) // 4
    psqt = int(ps[stm][bucket] - ps[1 - stm][bucket])
    psqt = int(psqt / 2)  # C truncation
    fc0 = a["b0"][bucket].astype(np.int64) + a["w0"][bucket].astype(np.int64) @ x
    in1 = np.zeros(32, dtype=np.int64)
    in1[:15] = np.minimum(127, (fc0[:15] * fc0[:15]) >> 19)
    in1[15:30] = np.clip(fc0[:15] >> 6, 0, 127)
    fc1 = np.clip((a["b1"][bucket].astype(np.int64) + a["w1"][bucket].astype(np.int64) @ in1) >> 6, 0, 127)
    fc2 = int(a["b2"][bucket][0] + a["w2"][bucket].astype(np.int64) @ fc1)
    fwd = int(fc0[15] * 9600 / 8128) if fc0[15] >= 0 else -int(-fc0[15] * 9600 / 8128)
    pos = fc2 + fwd
    trunc = lambda v: int(v / 16) if v >= 0 else -int(-v / 16)
    return trunc(psqt), trunc(pos)


@pytest.mark.parametrize("stress", [False, True])
def test_numpy_restatement_agrees(oracle_lib, stress):
    from fishnet_amd import synthnet
    seed = 7 if stress else 2
    a = synthnet.synth_net_arrays(128, seed, stress)
    net = oracle_lib.Net(synthnet.cached_synth_net(128, seed, stress))
    fens = [l.strip() for l in open(os.path.join(HERE, "golden", "special_fens.txt"))
            if l.strip() and not l.startswith("#")]
    for fen in fens:
        assert oracle_lib.net_output(net, fen) == np_net_output(a, fen), fen


def test_net_parser_rejects_corruption(oracle_lib, synth_small_path):
    data = open(synth_small_path, "rb").read()
    for bad in (data[:-1], data + b"\0", data[:4] + b"\1\2\3\4" + data[8:], b"\0" * 64):
        with pytest.raises(ValueError):
            oracle_lib.Net(data=bad)
    assert oracle_lib.Net(data=data).l1 == 128


@pytest.mark.parametrize("stress", [False, True])
def test_incremental_oracle_equals_refresh(oracle_lib, stress):
    """or_expand_eval_inc (children updated from the parent's accumulators, the CPU
    baseline's mode) gives exactly or_expand_eval's full refreshes, also when the int16
    accumulators wrap."""
    from fishnet_amd import synthnet
    small = oracle_lib.Net(synthnet.cached_synth_net(128, 7 if stress else 2, stress))
    big = oracle_lib.Net(synthnet.cached_synth_net(3072, 11 if stress else 1, stress))
    fens = [l.strip() for l in open(os.path.join(HERE, "golden", "special_fens.txt"))
            if l.strip() and not l.startswith("#")]
    for mode in (0, 1, 2):
        for fen in fens:
            a = oracle_lib.expand_eval(big, small, fen, mode)
            b = oracle_lib.expand_eval(big, small, fen, mode, incremental=True)
            assert a[0] == b[0] and a[1] == b[1] and np.array_equal(a[2], b[2]), (mode, fen)
        par, cnt, kids = oracle_lib.expand_eval_batch(big, small, fens, mode, True, threads=4, keep_children=True)
        for i, fen in enumerate(fens):
            p_exp, m_exp, k_exp = oracle_lib.expand_eval(big, small, fen, mode)
            assert tuple(par[i]) == p_exp and cnt[i] == len(m_exp) and np.array_equal(kids[i, :cnt[i]], k_exp)


def test_oracle_under_sanitizers(oracle_lib, tmp_path):
    """The oracle built with AddressSanitizer + UBSan (oracle/Makefile `sanitize`, a driver
    executable) over the hand-picked edge FENs plus a bad one: no sanitizer report, refresh
    and incremental expansion equal, and the same numbers as the regular build."""
    import shutil
    import subprocess
    from fishnet_amd import synthnet
    if not shutil.which("gcc"):
        pytest.skip("no host compiler")
    odir = os.path.join(HERE, "..", "oracle")
    r = subprocess.run(["make", "-s", "-C", odir, "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    exe = os.path.join(odir, "_build", "oracle_sanitize")
    fens = [ln.strip() for ln in open(os.path.join(HERE, "golden", "special_fens.txt"))
            if ln.strip() and not ln.startswith("#")][:12]
    fens.append("8/8/8/8/8/8/8/8 w - - 0 1")  # no kings: rejected
    fpath = tmp_path / "fens.txt"
    fpath.write_text("\n".join(fens) + "\n")
    big_p, small_p = synthnet.cached_synth_net(3072, 1), synthnet.cached_synth_net(128, 2)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, big_p, small_p, str(fpath)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.split("\n")
    big, small = oracle_lib.Net(big_p), oracle_lib.Net(small_p)
    for fen, line in zip(fens, lines):
        if line == "bad":
            with pytest.raises(ValueError):
                oracle_lib.perft(fen, 1)
            continue
        fv, fcp, n, s, p2 = (int(x) for x in line.split())
        e = oracle_lib.eval_fen(big, small, fen, oracle_lib.MODE_FULL)
        _, _, kids = oracle_lib.expand_eval(big, small, fen, oracle_lib.MODE_BIG)
        assert (fv, fcp) == (e[2], e[3]), fen
        assert (n, s) == (len(kids), int(kids["final_v"].astype(np.int64).sum())), fen
        assert p2 == oracle_lib.perft(fen, 2), fen
    assert lines[len(fens) - 1] == "bad"


# ---- the score rule (include/gpu_nnue.h at gn_eval; tests/golden/score_fens.json) -------
def _score_doc():
    return json.load(open(os.path.join(HERE, "golden", "score_fens.json")))


def test_score_goldens_regenerate_identically(oracle_lib, oracle_nets, synth_big_path, synth_small_path):
    g = _score_doc()
    sha = lambda p: hashlib.sha256(open(p, "rb").read()).hexdigest()
    assert g["nets"]["big"]["sha256"] == sha(synth_big_path)
    assert g["nets"]["small"]["sha256"] == sha(synth_small_path)
    big, small = oracle_nets
    for name, mode in (("full", 0), ("big", 1), ("small", 2)):
        rows = g["results"][name]
        got = oracle_lib.eval_fens(big, small, [r[0] for r in rows], mode, threads=4)
        assert [list(map(int, r)) for r in got.tolist()] == [r[1:] for r in rows]


def test_score_categories_mean_what_they_say(oracle_lib):
    """Each fixture category has the score fishnet would post: mate 0 / cp 0 without a legal
    move, a searched cp or mate in check, best_move a legal reply."""
    O = oracle_lib
    g = _score_doc()
    cats, cols = g["categories"], g["columns"]
    rec = {r[0]: dict(zip(cols[1:], r[1:])) for r in g["results"]["full"]}
    assert {k for k, v in cats.items() if v} == {"mate0", "stalemate", "searched_d1", "searched_d2", "mate+", "mate-"}
    for k, fens in cats.items():
        for fen in fens:
            r = rec[fen]
            moves = O.legal_moves(fen)
            if k in ("mate0", "stalemate"):
                assert not moves and r["flags"] & O.FLAG_NO_MOVES and r["score"] == 0 and r["best_move"] == 0
                assert bool(r["flags"] & O.FLAG_MATE) == (k == "mate0") == bool(r["flags"] & O.FLAG_IN_CHECK)
            else:
                assert moves and r["flags"] & O.FLAG_IN_CHECK and r["flags"] & O.FLAG_SEARCHED
                assert r["best_move"] in moves
                assert bool(r["flags"] & O.FLAG_MATE) == k.startswith("mate")
                if k == "mate+":
                    assert r["score"] >= 1
                if k == "mate-":
                    assert r["score"] <= -1


def py_rule_value(O, small, fen, depth):
    """Second restatement of the rule (negamax over oracle primitives, in Python)."""
    e = O.eval_fen(None, small, fen, O.MODE_SMALL)
    moves = O.legal_moves(fen)
    check = e[5] & O.FLAG_IN_CHECK
    if not moves:
        return (-32000 if check else 0), None
    if not check or depth == 0:
        return e[2], None
    best = None
    for m in sorted(moves):  # ties: the smaller move encoding (strict > keeps the first)
        v = -py_rule_value(O, small, O.child_fen(fen, m), depth - 1)[0]
        v = v - 1 if v >= 31754 else v + 1 if v <= -31754 else v
        if best is None or v > best[0]:
            best = (v, m)
    return best


def test_score_rule_restated_in_python(oracle_lib, oracle_nets):
    O = oracle_lib
    _, small = oracle_nets
    g = _score_doc()
    cols = g["columns"]
    for row in g["results"]["small"]:
        r = dict(zip(cols[1:], row[1:]))
        if not r["flags"] & O.FLAG_SEARCHED:
            continue
        v, m = py_rule_value(O, small, row[0], 2)
        assert m == r["best_move"], row[0]
        if r["flags"] & O.FLAG_MATE:
            ply = 32000 - abs(v)
            assert r["score"] == ((ply + 1) // 2 if v > 0 else -(ply // 2)), row[0]
        else:
            assert r["score"] == py_to_cp(v, row[0]), row[0]
