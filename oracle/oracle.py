"""ctypes wrapper over oracle/_build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It is the checker for the product path (libgpu_nnue.so); the
product never imports it.  See oracle.h for what is restated and the parity
status (perft pinned by public known answers; NNUE "parity unpinned").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
# the same source built -O3 -march=native (bench.py's cpu_baseline; integer-identical results)
NATIVE_LIB_PATH = os.path.join(HERE, "_build", "liboracle_native.so")

MODE_FULL, MODE_BIG, MODE_SMALL = 0, 1, 2
FLAG_IN_CHECK, FLAG_SMALLNET, FLAG_BAD_FEN, FLAG_REEVAL = 1, 2, 4, 8
FLAG_MATE, FLAG_NO_SCORE, FLAG_SEARCHED, FLAG_NO_MOVES = 32, 64, 128, 256


class OrEval(C.Structure):
    _fields_ = [("psqt", C.c_int32), ("positional", C.c_int32), ("final_v", C.c_int32),
                ("final_cp", C.c_int32), ("score", C.c_int32), ("flags", C.c_uint16), ("best_move", C.c_uint16)]


EVAL_DTYPE = np.dtype([("psqt", "<i4"), ("positional", "<i4"), ("final_v", "<i4"), ("final_cp", "<i4"),
                       ("score", "<i4"), ("flags", "<u2"), ("best_move", "<u2")])
assert EVAL_DTYPE.itemsize == C.sizeof(OrEval) == 24


def _tup(e):
    return (e.psqt, e.positional, e.final_v, e.final_cp, e.score, e.flags, e.best_move)

_lib = None


def build(native=False):
    subprocess.run(["make", "-s", "-C", HERE] + (["native"] if native else []), check=True)


def use_library(path):
    """Switch the oracle to another build of the same source (Net objects made before stay
    valid: same struct layout, same libc allocator)."""
    global _lib, LIB_PATH
    LIB_PATH, _lib = path, None
    return lib()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build(native=LIB_PATH == NATIVE_LIB_PATH)
        L = C.CDLL(LIB_PATH)
        L.or_net_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.or_net_load_mem.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
        L.or_net_free.argtypes = [C.c_void_p]
        L.or_net_l1.argtypes = [C.c_void_p]
        L.or_net_hash.argtypes = [C.c_void_p]
        L.or_net_hash.restype = C.c_uint32
        L.or_expected_hash.argtypes = [C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.or_expected_hash.restype = C.c_uint32
        L.or_eval_fen.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, C.c_int, C.POINTER(OrEval)]
        L.or_eval_fens.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_char_p), C.c_size_t,
                                   C.c_int, C.c_void_p, C.c_int]
        L.or_features.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_uint32), C.c_int]
        L.or_accumulate.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_void_p, C.c_void_p]
        L.or_net_output.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.or_legal_moves.argtypes = [C.c_char_p, C.POINTER(C.c_uint16), C.c_int]
        L.or_child_fen.argtypes = [C.c_char_p, C.c_uint16, C.c_char_p, C.c_int]
        L.or_normalize_fen.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.or_perft.argtypes = [C.c_char_p, C.c_int]
        L.or_perft.restype = C.c_uint64
        L.or_expand_eval.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, C.c_int, C.POINTER(OrEval),
                                     C.POINTER(C.c_uint16), C.c_void_p, C.c_int]
        L.or_expand_eval_inc.argtypes = L.or_expand_eval.argtypes
        L.or_expand_eval_batch.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_char_p), C.c_size_t, C.c_int,
                                           C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


class Net:
    """A loaded .nnue network (oracle side)."""

    def __init__(self, path=None, data: bytes | None = None):
        err = C.create_string_buffer(256)
        h = C.c_void_p()
        if data is not None:
            buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
            rc = lib().or_net_load_mem(buf, len(data), C.byref(h), err, 256)
        else:
            rc = lib().or_net_load(str(path).encode(), C.byref(h), err, 256)
        if rc != 0:
            raise ValueError(f"oracle net load failed: {err.value.decode()}")
        self.h = h

    @property
    def l1(self):
        return lib().or_net_l1(self.h)

    @property
    def hash(self):
        return lib().or_net_hash(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_net_free(self.h)
            self.h = None


def expected_hash(l1):
    ft, arch = C.c_uint32(), C.c_uint32()
    h = lib().or_expected_hash(l1, C.byref(ft), C.byref(arch))
    return h, ft.value, arch.value


def _h(net):
    return net.h if net is not None else None


def eval_fen(big, small, fen, mode=MODE_FULL):
    out = OrEval()
    lib().or_eval_fen(_h(big), _h(small), fen.encode(), mode, C.byref(out))
    return _tup(out)


def eval_fens(big, small, fens, mode=MODE_FULL, threads=1):
    n = len(fens)
    arr = (C.c_char_p * n)(*[f.encode() for f in fens])
    out = np.zeros(n, dtype=EVAL_DTYPE)
    lib().or_eval_fens(_h(big), _h(small), arr, n, mode, out.ctypes.data, threads)
    return out


def features(fen, perspective):
    buf = (C.c_uint32 * 64)()
    n = lib().or_features(fen.encode(), perspective, buf, 64)
    if n < 0:
        raise ValueError("bad fen")
    return list(buf[:n])


def accumulate(net, fen, perspective):
    acc = np.zeros(net.l1, dtype=np.int16)
    ps = np.zeros(8, dtype=np.int32)
    if lib().or_accumulate(net.h, fen.encode(), perspective, acc.ctypes.data, ps.ctypes.data):
        raise ValueError("bad fen")
    return acc, ps


def net_output(net, fen):
    a, b = C.c_int32(), C.c_int32()
    if lib().or_net_output(net.h, fen.encode(), C.byref(a), C.byref(b)):
        raise ValueError("bad fen")
    return a.value, b.value


def legal_moves(fen):
    buf = (C.c_uint16 * 256)()
    n = lib().or_legal_moves(fen.encode(), buf, 256)
    if n < 0:
        raise ValueError("bad fen")
    return list(buf[:n])


def child_fen(fen, move):
    out = C.create_string_buffer(128)
    if lib().or_child_fen(fen.encode(), move, out, 128) < 0:
        raise ValueError("bad fen")
    return out.value.decode()


def normalize_fen(fen):
    out = C.create_string_buffer(128)
    if lib().or_normalize_fen(fen.encode(), out, 128) < 0:
        raise ValueError("bad fen")
    return out.value.decode()


def perft(fen, depth):
    v = lib().or_perft(fen.encode(), depth)
    if v == 2**64 - 1:
        raise ValueError("bad fen")
    return v


def expand_eval(big, small, fen, mode=MODE_FULL, incremental=False):
    parent = OrEval()
    moves = (C.c_uint16 * 256)()
    kids = np.zeros(256, dtype=EVAL_DTYPE)
    f = lib().or_expand_eval_inc if incremental else lib().or_expand_eval
    n = f(_h(big), _h(small), fen.encode(), mode, C.byref(parent), moves, kids.ctypes.data, 256)
    if n < 0:
        raise ValueError("bad fen")
    return _tup(parent), list(moves[:n]), kids[:n].copy()


def expand_eval_batch(big, small, fens, mode=MODE_FULL, incremental=True, threads=1, keep_children=False):
    """n parents + all children on `threads` C threads: (parents[n], child_counts[n], children[n, 256] or None)."""
    n = len(fens)
    arr = (C.c_char_p * n)(*[f.encode() for f in fens])
    parents = np.zeros(n, dtype=EVAL_DTYPE)
    counts = np.zeros(n, dtype=np.int32)
    kids = np.zeros((n, 256), dtype=EVAL_DTYPE) if keep_children else None
    lib().or_expand_eval_batch(_h(big), _h(small), arr, n, mode, int(incremental), threads, parents.ctypes.data,
                               counts.ctypes.data, None if kids is None else kids.ctypes.data)
    return parents, counts, kids


def move_to_uci(m):
    """Stockfish move encoding -> UCI text (Chess960 castling: king takes rook)."""
    to, frm, typ = m & 63, (m >> 6) & 63, m >> 14
    sq = lambda s: "abcdefgh"[s & 7] + str((s >> 3) + 1)
    u = sq(frm) + sq(to)
    if typ == 1:
        u += "nbrq"[(m >> 12) & 3]
    return u


# ---- lichess batch replay (restatement for tests) --------------------------
# IncomingBatch::from_acquired (/root/reference/src/queue.rs:548-700) replays
# root_fen + the batch's UCI moves with shakmaty 0.27.3 (UciMove::to_move,
# queue.rs:576; play_unchecked, queue.rs:578).  shakmaty is a Rust crate that is
# not vendored in /root/reference (Cargo.lock pins 0.27.3); its published
# to_move rule is restated here on top of this oracle's own movegen:
#   king onto a square of the castling rights        -> castling with that rook;
#   king e1/e8 -> c/g file of its back rank            -> castling with the a/h rook;
#   otherwise from/to (+ promotion letter n/b/r/q)    -> must be a legal move.

class IllegalMove(ValueError):
    def __init__(self, index, uci):
        super().__init__(f"move {index} ({uci}) is not legal")
        self.index, self.uci = index, uci


def _sq(s):
    if len(s) != 2 or s[0] not in "abcdefgh" or s[1] not in "12345678":
        return None
    return (ord(s[1]) - ord("1")) * 8 + ord(s[0]) - ord("a")


def _placement(fen):
    board, rank, file = {}, 7, 0
    for ch in fen.split()[0]:
        if ch == "/":
            rank, file = rank - 1, 0
        elif ch.isdigit():
            file += int(ch)
        else:
            board[rank * 8 + file] = ch
            file += 1
    return board


def castling_rook_squares(fen):
    """Rook squares carrying castling rights (X-FEN / Shredder, as normalize_fen prints them)."""
    board, field, out = _placement(fen), fen.split()[2], set()
    for ch in field:
        if ch == "-":
            continue
        white = ch.isupper()
        base = 0 if white else 56
        rook, king = ("R", "K") if white else ("r", "k")
        ksq = next((s for s in range(base, base + 8) if board.get(s) == king), None)
        rooks = [s for s in range(base, base + 8) if board.get(s) == rook]
        u = ch.upper()
        if u == "K":
            cand = [s for s in rooks if ksq is not None and s > ksq]
            if cand:
                out.add(max(cand))
        elif u == "Q":
            cand = [s for s in rooks if ksq is not None and s < ksq]
            if cand:
                out.add(min(cand))
        else:
            out.add(base + ord(u) - ord("A"))
    return out


def uci_to_move(fen, uci):
    """shakmaty UciMove::to_move on this oracle's movegen; None when not legal."""
    if len(uci) not in (4, 5):
        return None
    frm, to = _sq(uci[0:2]), _sq(uci[2:4])
    if frm is None or to is None:
        return None
    promo = uci[4] if len(uci) == 5 else None
    if promo is not None and promo not in "nbrq":
        return None
    board = _placement(fen)
    pc = board.get(frm)
    if pc is None or (promo and pc.upper() != "P"):
        return None
    white = fen.split()[1] == "w"
    rook = None
    if pc.upper() == "K":
        if to in castling_rook_squares(fen):
            rook = to
        elif frm == (4 if white else 60) and to // 8 == (0 if white else 7) and to % 8 in (2, 6):
            rook = (to & 56) | (0 if to % 8 == 2 else 7)
    for m in legal_moves(fen):
        mt, mf, typ = m & 63, (m >> 6) & 63, m >> 14
        if mf != frm:
            continue
        if rook is not None:
            if typ == 3 and mt == rook:
                return m
            continue
        if typ == 3 or mt != to:
            continue
        if typ == 1:
            if promo != "nbrq"[(m >> 12) & 3]:
                continue
        elif promo:
            continue
        return m
    return None


def replay_game(root_fen, moves):
    """-> (fens of positions 0..=len, played moves in Stockfish encoding); raises IllegalMove."""
    fen = normalize_fen(root_fen)
    fens, played = [fen], []
    for i, u in enumerate(moves.split() if isinstance(moves, str) else moves):
        m = uci_to_move(fen, u)
        if m is None:
            raise IllegalMove(i + 1, u)
        fen = child_fen(fen, m)
        fens.append(fen)
        played.append(m)
    return fens, played
