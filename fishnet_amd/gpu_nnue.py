"""Python host mirror of the `gpu_nnue` module fishnet would call (ctypes over
libgpu_nnue.so, include/gpu_nnue.h).

The reference's engine plugin API is `StockfishStub::go_multiple(Chunk)`
(/root/reference/src/stockfish.rs:36-47); the north-star `gpu_nnue` module adds
`load_net(.nnue)` and `evaluate_batch(&[Fen]) -> Vec<(psqt, positional, final)>`
beside it.  This module exposes exactly those two plus expansion, perft and the
device-resident entry points used by bench.py.  There is no CPU fallback: if
the HIP library is missing or no gfx950 device is present, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPU_NNUE_LIB", os.path.join(HERE, "lib", "libgpu_nnue.so"))

MODE_FULL, MODE_BIG, MODE_SMALL = 0, 1, 2
FLAG_IN_CHECK, FLAG_SMALLNET, FLAG_BAD_FEN, FLAG_REEVAL, FLAG_SKIPPED = 1, 2, 4, 8, 16
FLAG_MATE, FLAG_NO_SCORE, FLAG_SEARCHED, FLAG_NO_MOVES = 32, 64, 128, 256
ERRORS = {-1: "INVALID", -2: "IO", -3: "FORMAT", -4: "HIP", -5: "NOMEM", -6: "CAPACITY",
          -7: "NODEVICE", -8: "NONET", -9: "ILLEGAL_MOVE"}
E_INVALID, E_IO, E_FORMAT, E_HIP, E_NOMEM, E_CAPACITY, E_NODEVICE, E_NONET, E_ILLEGAL_MOVE = -1, -2, -3, -4, -5, -6, -7, -8, -9

# gn_eval (ABI v3): the static evaluation, and the score fishnet posts (gpu_nnue.h)
EVAL_DTYPE = np.dtype([("psqt", "<i4"), ("positional", "<i4"), ("final_v", "<i4"), ("final_cp", "<i4"),
                       ("score", "<i4"), ("flags", "<u2"), ("best_move", "<u2")])
BOARD_DTYPE = np.dtype([("occ", "<u8"), ("pc", "u1", (16,)), ("stm_ep", "u1"), ("reserved", "u1"),
                        ("castle", "<u2"), ("rule50", "<u2"), ("fullmove", "<u2")])
# gn_child (ABI v4): a legal child's record from the host-buffer expansion calls, 12 bytes:
# final_cp (signed 24 bits) and the low 8 flag bits share cp_flags (gpu_nnue.h at gn_child)
CHILD_DTYPE = np.dtype([("psqt", "<i4"), ("positional", "<i4"), ("cp_flags", "<i4")])
# ... and decoded (decode_children / children_from_evals), the form the tests compare
CHILD_VIEW_DTYPE = np.dtype([("psqt", "<i4"), ("positional", "<i4"), ("final_cp", "<i4"), ("flags", "<u2")])
EVAL_SIZE, BOARD_SIZE, CHILD_SIZE = EVAL_DTYPE.itemsize, BOARD_DTYPE.itemsize, CHILD_DTYPE.itemsize
assert EVAL_SIZE == 24 and BOARD_SIZE == 32 and CHILD_SIZE == 12
ABI_VERSION = 4

EXPORTS = ["gn_load_net", "gn_load_net_memory", "gn_free", "gn_last_error", "gn_abi_version",
           "gn_get_eval_params", "gn_set_eval_params", "gn_net_info", "gn_evaluate_batch",
           "gn_evaluate_batch_mode", "gn_expand_and_evaluate", "gn_perft", "gn_pack_fens",
           "gn_board_to_fen", "gn_random_positions", "gn_evaluate_device", "gn_expand_device",
           "gn_device_alloc", "gn_device_free", "gn_memcpy_h2d", "gn_memcpy_d2h", "gn_synchronize",
           "gn_time_evaluate_device", "gn_random_positions_device", "gn_set_option", "gn_get_option",
           "gn_time_expand_device", "gn_random_games_device", "gn_replay_game", "gn_evaluate_games",
           "gn_net_sha256", "gn_partition", "gn_checksum_device",
           "gn_boards_to_fens", "gn_load_net_archive", "gn_archive_read", "gn_expand2_device",
           "gn_random_games_uci"]
OPT_INCREMENTAL_CHILDREN, OPT_XCD_SWIZZLE, OPT_KING_SORT, OPT_CHAIN, OPT_KING_CACHE = 1, 2, 3, 4, 5
OPT_CHUNK_PARENTS, OPT_COALESCE, OPT_STREAM_SLICES, OPT_FAST_BATCH, OPT_EXPAND_PIPELINE = 6, 7, 8, 9, 10
STAT_PLAN_NS, STAT_STREAM_NS, STAT_SCRATCH_PADS, STAT_FINISH_NS = 101, 102, 103, 104
STAT_BATCH_LAUNCHES, STAT_BATCH_CALLS, STAT_FAST_BATCHES, STAT_FAST_FALLBACKS = 117, 118, 119, 120
HOST_STAGES = {"parse": 110, "upload": 111, "replay": 112, "compute": 113, "download": 114, "tail": 115, "total": 116}
EXPAND_STAGES = ["count_scan", "total_readback", "write_children", "classify", "small_net", "big_net", "finalize",
                 "score"]


def decode_children(raw) -> np.ndarray:
    """gn_child records -> CHILD_VIEW_DTYPE (psqt, positional, final_cp, flags)."""
    raw = np.asarray(raw, dtype=CHILD_DTYPE)
    out = np.empty(raw.shape, dtype=CHILD_VIEW_DTYPE)
    cf = raw["cp_flags"].astype(np.int64)
    out["psqt"], out["positional"] = raw["psqt"], raw["positional"]
    out["final_cp"] = ((cf & 0xFFFFFF) ^ 0x800000) - 0x800000
    out["flags"] = (cf >> 24) & 0xFF
    return out


def children_from_evals(ev) -> np.ndarray:
    """gn_eval child records (the device-resident calls, the oracle) -> the fields a gn_child keeps,
    as CHILD_VIEW_DTYPE: psqt, positional, final_cp and the low 8 flag bits."""
    ev = np.asarray(ev, dtype=EVAL_DTYPE)
    out = np.empty(ev.shape, dtype=CHILD_VIEW_DTYPE)
    out["psqt"], out["positional"], out["final_cp"] = ev["psqt"], ev["positional"], ev["final_cp"]
    out["flags"] = ev["flags"] & 0xFF
    return out


class GnError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gpu_nnue error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class EvalParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "small_net_threshold", "psqt_weight", "positional_weight", "reeval_threshold",
        "complexity_div_small", "complexity_div_big", "material_pawn_small", "material_pawn_big",
        "material_base", "rule50_div", "value_clamp")] + [
        ("piece_value", C.c_int32 * 5), ("wdl_a", C.c_double * 4), ("wdl_material_min", C.c_int32),
        ("wdl_material_max", C.c_int32), ("wdl_material_anchor", C.c_int32), ("wdl_piece_weight", C.c_int32 * 5)]


class GnGame(C.Structure):
    """gn_game: one acquired lichess batch (root FEN, UCI moves string, skipPositions)."""
    _fields_ = [("root_fen", C.c_char_p), ("uci_moves", C.c_char_p),
                ("skip_positions", C.POINTER(C.c_uint32)), ("n_skip", C.c_size_t)]


def _games_array(games):
    """[(root_fen, moves, skip)] -> (gn_game array, keep-alive list).  moves: str or list of UCI."""
    keep, arr = [], (GnGame * max(len(games), 1))()
    for i, g in enumerate(games):
        root, moves, skip = (tuple(g) + ((),) * 3)[:3]
        mv = moves if isinstance(moves, str) else " ".join(moves or ())
        sk = (C.c_uint32 * max(len(skip), 1))(*skip)
        keep += [root.encode(), mv.encode(), sk]
        arr[i].root_fen, arr[i].uci_moves = keep[-3], keep[-2]
        arr[i].skip_positions = C.cast(sk, C.POINTER(C.c_uint32))
        arr[i].n_skip = len(skip)
    return arr, keep


_lib = None


def lib():
    """Loads libgpu_nnue.so (never falls back to anything else)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgpu_nnue.so not built at {LIB_PATH}: run `python -m fishnet_amd.build`")
    L = C.CDLL(LIB_PATH)
    vp, sz, i32 = C.c_void_p, C.c_size_t, C.c_int
    sig = {
        "gn_load_net": [C.c_char_p, C.c_char_p, vp, i32, C.POINTER(vp)],
        "gn_load_net_memory": [vp, sz, vp, sz, vp, i32, C.POINTER(vp)],
        "gn_free": [vp],
        "gn_last_error": [],
        "gn_abi_version": [],
        "gn_get_eval_params": [vp, C.POINTER(EvalParams)],
        "gn_set_eval_params": [vp, C.POINTER(EvalParams)],
        "gn_net_info": [vp, C.POINTER(i32), C.POINTER(C.c_uint32), C.POINTER(i32), C.POINTER(C.c_uint32)],
        "gn_evaluate_batch": [vp, vp, sz, vp],
        "gn_evaluate_batch_mode": [vp, vp, sz, i32, vp],
        "gn_expand_and_evaluate": [vp, vp, sz, i32, vp, vp, vp, vp, sz],
        "gn_perft": [vp, C.c_char_p, i32, C.POINTER(C.c_uint64)],
        "gn_pack_fens": [vp, sz, vp, vp],
        "gn_board_to_fen": [vp, C.c_char_p, sz],
        "gn_random_positions": [C.c_uint64, sz, sz, i32, vp],
        "gn_evaluate_device": [vp, i32, vp, sz, i32, vp, vp],
        "gn_expand_device": [vp, i32, vp, sz, i32, vp, vp, vp, vp, vp, sz, C.POINTER(sz), vp],
        "gn_device_alloc": [vp, i32, sz, C.POINTER(vp)],
        "gn_device_free": [vp, i32, vp],
        "gn_memcpy_h2d": [vp, i32, vp, vp, sz],
        "gn_memcpy_d2h": [vp, i32, vp, vp, sz],
        "gn_synchronize": [vp, i32],
        "gn_time_evaluate_device": [vp, i32, vp, sz, i32, vp, i32, C.POINTER(C.c_float), vp, C.POINTER(C.c_uint64)],
        "gn_checksum_device": [vp, i32, vp, sz, C.POINTER(C.c_uint64)],
        "gn_random_positions_device": [vp, i32, C.c_uint64, sz, sz, i32, vp, vp],
        "gn_set_option": [vp, i32, C.c_int64],
        "gn_get_option": [vp, i32, C.POINTER(C.c_int64)],
        "gn_time_expand_device": [vp, i32, vp, sz, i32, i32, C.POINTER(C.c_float), C.POINTER(sz), vp,
                                  C.POINTER(C.c_uint64), vp, vp, vp, vp, sz],
        "gn_random_games_device": [vp, i32, C.c_uint64, sz, sz, i32, vp, vp],
        "gn_replay_game": [C.POINTER(GnGame), vp, vp, vp, sz, C.POINTER(sz)],
        "gn_net_sha256": [vp, sz, C.c_char_p],
        "gn_partition": [vp, sz, i32, vp],
        "gn_boards_to_fens": [vp, sz, vp, sz],
        "gn_evaluate_games": [vp, vp, sz, i32, i32, vp, vp, vp, sz, vp, vp, vp, sz],
        "gn_load_net_archive": [C.c_char_p, C.c_char_p, C.c_char_p, vp, i32, C.POINTER(vp)],
        "gn_archive_read": [C.c_char_p, C.c_char_p, vp, sz, C.POINTER(sz)],
        "gn_expand2_device": [vp, i32, vp, sz, i32, vp, vp, vp, vp, vp, sz, vp, vp, vp, sz, C.POINTER(sz),
                              C.POINTER(sz), vp],
        "gn_random_games_uci": [C.c_uint64, sz, sz, i32, vp, sz],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = i32
    L.gn_free.restype = None
    L.gn_last_error.restype = C.c_char_p
    if L.gn_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {L.gn_abi_version()}, this module expects {ABI_VERSION}: rebuild it")
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise GnError(rc, (lib().gn_last_error() or b"").decode(errors="replace"))


def _fen_array(fens):
    enc = [f.encode() for f in fens]
    arr = (C.c_char_p * len(enc))(*enc)
    return arr, enc


def pack_fens(fens):
    """FEN strings -> (boards[BOARD_DTYPE], ok[bool]); host only, no GPU needed."""
    n = len(fens)
    boards = np.zeros(n, dtype=BOARD_DTYPE)
    ok = np.zeros(n, dtype=np.uint8)
    arr, _keep = _fen_array(fens)
    _check(lib().gn_pack_fens(arr, n, boards.ctypes.data, ok.ctypes.data))
    return boards, ok.astype(bool)


def board_to_fen(board) -> str:
    b = np.ascontiguousarray(np.asarray(board, dtype=BOARD_DTYPE).reshape(1))
    buf = C.create_string_buffer(128)
    _check(lib().gn_board_to_fen(b.ctypes.data, buf, 128))
    return buf.value.decode()


def boards_to_fens(boards) -> list:
    """FENs of many boards at once (gn_boards_to_fens, multithreaded C)."""
    b = np.ascontiguousarray(np.asarray(boards, dtype=BOARD_DTYPE).reshape(-1))
    buf = np.zeros((len(b), 100), dtype=np.uint8)
    _check(lib().gn_boards_to_fens(b.ctypes.data, len(b), buf.ctypes.data, 100))
    return [bytes(r[:np.argmin(r)]).decode() for r in buf] if len(b) else []


def random_positions(seed: int, first: int, n: int, max_plies: int = 160):
    boards = np.zeros(n, dtype=BOARD_DTYPE)
    _check(lib().gn_random_positions(seed, first, n, max_plies, boards.ctypes.data))
    return boards


def replay_game(root_fen: str, moves, skip=()):
    """IncomingBatch::from_acquired replay (host only): (boards[n+1], skipped[n+1], moves[n] Stockfish encoding)."""
    arr, _keep = _games_array([(root_fen, moves, tuple(skip))])
    n = C.c_size_t()
    rc = lib().gn_replay_game(arr, None, None, None, 0, C.byref(n))
    if rc not in (0, E_CAPACITY):
        _check(rc)
    cap = n.value
    boards = np.zeros(cap, dtype=BOARD_DTYPE)
    skipped = np.zeros(cap, dtype=np.uint8)
    mv = np.zeros(max(cap - 1, 1), dtype=np.uint16)
    _check(lib().gn_replay_game(arr, boards.ctypes.data, skipped.ctypes.data, mv.ctypes.data, cap, C.byref(n)))
    return boards, skipped.astype(bool), mv[:cap - 1]


def random_games_uci(seed: int, first_game: int, n_games: int, plies: int = 80) -> list:
    """UCI move strings of the games gn_random_games_device plays (lichess wire form)."""
    stride = 6 * plies + 1
    buf = np.zeros((n_games, stride), dtype=np.uint8)
    _check(lib().gn_random_games_uci(seed, first_game, n_games, plies, buf.ctypes.data, stride))
    return [bytes(r[:np.argmin(r)]).decode() for r in buf]


def net_sha256(data: bytes) -> str:
    """gn_net_sha256: hex SHA-256 (Stockfish net names are nn-<first 12 digits>.nnue)."""
    out = C.create_string_buffer(65)
    buf = (C.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    _check(lib().gn_net_sha256(buf, len(data), out))
    return out.value.decode()


def partition(n_items: int, n_shards: int, weights=None):
    """gn_partition: bounds[n_shards + 1] of contiguous shards (the library's and bench's one partitioner)."""
    b = np.zeros(n_shards + 1, dtype=np.uint64)
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.uint32)
    _check(lib().gn_partition(None if w is None else w.ctypes.data, n_items, n_shards, b.ctypes.data))
    return [int(x) for x in b]


def default_eval_params() -> EvalParams:
    p = EvalParams()
    _check(lib().gn_get_eval_params(None, C.byref(p)))
    return p


class DeviceBuffer:
    def __init__(self, ctx: "GpuNnue", nbytes: int, slot: int = 0):
        self.ctx, self.slot, self.nbytes = ctx, slot, nbytes
        self.ptr = C.c_void_p()
        _check(lib().gn_device_alloc(ctx.h, slot, nbytes, C.byref(self.ptr)))

    @property
    def addr(self):
        return self.ptr.value

    def upload(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        _check(lib().gn_memcpy_h2d(self.ctx.h, self.slot, self.ptr, a.ctypes.data, a.nbytes))

    def download(self, dtype, count, offset=0):
        """count elements of dtype starting at element `offset`."""
        out = np.empty(count, dtype=dtype)
        if count:
            src = C.c_void_p(self.addr + offset * np.dtype(dtype).itemsize)
            assert (offset + count) * np.dtype(dtype).itemsize <= self.nbytes
            _check(lib().gn_memcpy_d2h(self.ctx.h, self.slot, out.ctypes.data, src, out.nbytes))
        return out

    def free(self):
        if self.ptr and self.ptr.value:
            lib().gn_device_free(self.ctx.h, self.slot, self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceView(DeviceBuffer):
    """Device memory the library does not own (a torch tensor's storage, e.g. for RCCL): the
    same upload / download / pointer interface as DeviceBuffer; never freed here."""

    def __init__(self, ctx: "GpuNnue", tensor, slot: int = 0):
        self.ctx, self.slot, self.tensor = ctx, slot, tensor
        self.nbytes = tensor.numel() * tensor.element_size()
        self.ptr = C.c_void_p(tensor.data_ptr())

    def free(self):
        self.ptr = C.c_void_p()


def archive_read(path, member):
    """One member of an assets archive (zstd + ar) as bytes (gn_archive_read; CPU only)."""
    size = C.c_size_t()
    rc = lib().gn_archive_read(path.encode(), member.encode(), None, 0, C.byref(size))
    if rc not in (0, E_CAPACITY):
        _check(rc)
    buf = (C.c_uint8 * max(size.value, 1))()
    _check(lib().gn_archive_read(path.encode(), member.encode(), buf, size.value, C.byref(size)))
    return bytes(buf[:size.value])


class GpuNnue:
    """load_net + evaluate_batch (the north-star `gpu_nnue` module surface)."""

    def __init__(self, big_path=None, small_path=None, devices=None, big_bytes=None, small_bytes=None,
                 archive=None, big_member=None, small_member=None):
        self.h = C.c_void_p()
        devs = (C.c_int * len(devices))(*devices) if devices else None
        nd = len(devices) if devices else 0
        if archive is not None:  # fishnet's assets.ar.zst (gn_load_net_archive)
            enc = lambda x: x.encode() if x else None
            _check(lib().gn_load_net_archive(archive.encode(), enc(big_member), enc(small_member), devs, nd,
                                             C.byref(self.h)))
        elif big_bytes is not None or small_bytes is not None:
            bb = (C.c_uint8 * len(big_bytes)).from_buffer_copy(big_bytes) if big_bytes is not None else None
            sb = (C.c_uint8 * len(small_bytes)).from_buffer_copy(small_bytes) if small_bytes is not None else None
            _check(lib().gn_load_net_memory(bb, len(big_bytes or b""), sb, len(small_bytes or b""), devs, nd,
                                            C.byref(self.h)))
        else:
            _check(lib().gn_load_net(big_path.encode() if big_path else None,
                                     small_path.encode() if small_path else None, devs, nd, C.byref(self.h)))

    def close(self):
        if self.h and self.h.value:
            lib().gn_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def net_info(self):
        a, c = C.c_int(), C.c_int()
        b, d = C.c_uint32(), C.c_uint32()
        _check(lib().gn_net_info(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"big_l1": a.value, "big_hash": b.value, "small_l1": c.value, "small_hash": d.value}

    def eval_params(self) -> EvalParams:
        p = EvalParams()
        _check(lib().gn_get_eval_params(self.h, C.byref(p)))
        return p

    def set_eval_params(self, p: EvalParams):
        _check(lib().gn_set_eval_params(self.h, C.byref(p)))

    def evaluate_batch(self, fens, mode=MODE_FULL) -> np.ndarray:
        n = len(fens)
        out = np.zeros(n, dtype=EVAL_DTYPE)
        arr, _keep = _fen_array(fens)
        _check(lib().gn_evaluate_batch_mode(self.h, arr, n, mode, out.ctypes.data))
        return out

    def expand_and_evaluate(self, fens, mode=MODE_FULL, cap=None):
        """gn_expand_and_evaluate: (parent gn_eval records, child offsets, child moves, children as
        CHILD_VIEW_DTYPE decoded from the library's gn_child records)."""
        n = len(fens)
        arr, _keep = _fen_array(fens)
        offsets = np.zeros(n + 1, dtype=np.uint32)
        parents = np.zeros(n, dtype=EVAL_DTYPE)
        cap = cap if cap is not None else 64 * n + 256
        for _ in range(2):
            moves = np.zeros(max(cap, 1), dtype=np.uint16)
            kids = np.zeros(max(cap, 1), dtype=CHILD_DTYPE)
            rc = lib().gn_expand_and_evaluate(self.h, arr, n, mode, parents.ctypes.data, offsets.ctypes.data,
                                              moves.ctypes.data, kids.ctypes.data, cap)
            if rc == -6 and int(offsets[-1]) > cap:
                cap = int(offsets[-1])
                continue
            _check(rc)
            t = int(offsets[-1])
            return parents, offsets, moves[:t], decode_children(kids[:t])
        raise GnError(-6, "capacity retry failed")

    def evaluate_games(self, games, mode=MODE_FULL, children=False):
        """gn_evaluate_games over [(root_fen, moves, skip)]: per game a dict with status, evals of
        positions 0..=moves (skipped ones flagged FLAG_SKIPPED) and, with children, per position
        (child moves, children as CHILD_VIEW_DTYPE)."""
        arr, _keep = _games_array(games)
        ng = len(games)
        offs = np.zeros(ng + 1, dtype=np.uint32)
        status = np.zeros(max(ng, 1), dtype=np.int32)
        pcap, ccap = 0, 0
        for _ in range(3):
            pos = np.zeros(max(pcap, 1), dtype=EVAL_DTYPE)
            coffs = np.zeros(pcap + 1, dtype=np.uint32)
            cmv = np.zeros(max(ccap, 1), dtype=np.uint16)
            cev = np.zeros(max(ccap, 1), dtype=CHILD_DTYPE)
            rc = lib().gn_evaluate_games(self.h, arr, ng, mode, int(children), offs.ctypes.data, status.ctypes.data,
                                         pos.ctypes.data, pcap, coffs.ctypes.data if children else None,
                                         cmv.ctypes.data, cev.ctypes.data, ccap)
            if rc == E_CAPACITY:
                need_p = int(offs[-1])
                need_c = int(coffs[-1]) if children and need_p <= pcap else ccap
                pcap, ccap = max(pcap, need_p), max(ccap, need_c)
                continue
            _check(rc)
            cev = decode_children(cev)
            out = []
            for g in range(ng):
                a, b = int(offs[g]), int(offs[g + 1])
                d = {"status": int(status[g]), "evals": pos[a:b].copy()}
                if children:
                    d["children"] = [(cmv[coffs[i]:coffs[i + 1]].copy(), cev[coffs[i]:coffs[i + 1]].copy())
                                     for i in range(a, b)]
                out.append(d)
            return out
        raise GnError(E_CAPACITY, "capacity retry failed")

    def evaluate_games_arrays(self, arr, ng, mode=MODE_FULL, children=True, caps=None, bufs=None):
        """gn_evaluate_games on a prepared gn_game array (_games_array), results as flat arrays:
        (position_offsets, game_status, positions, child_offsets, child_moves, children, caps);
        children are the library's raw gn_child records (CHILD_DTYPE; decode_children).
        caps = (position_cap, child_cap) from an earlier call avoid the sizing retry; bufs (a dict,
        filled on first use) keeps the output arrays for the next call (a caller's reused buffers)."""
        pcap, ccap = caps or (0, 0)
        bufs = {} if bufs is None else bufs
        offs = np.zeros(ng + 1, dtype=np.uint32)
        status = np.zeros(max(ng, 1), dtype=np.int32)
        for _ in range(3):
            if bufs.get("caps") != (pcap, ccap):
                bufs.update(caps=(pcap, ccap), pos=np.empty(max(pcap, 1), dtype=EVAL_DTYPE),
                            coffs=np.empty(pcap + 1, dtype=np.uint32), cmv=np.empty(max(ccap, 1), dtype=np.uint16),
                            cev=np.empty(max(ccap, 1), dtype=CHILD_DTYPE))
            pos, coffs, cmv, cev = bufs["pos"], bufs["coffs"], bufs["cmv"], bufs["cev"]
            rc = lib().gn_evaluate_games(self.h, arr, ng, mode, int(children), offs.ctypes.data, status.ctypes.data,
                                         pos.ctypes.data, pcap, coffs.ctypes.data if children else None,
                                         cmv.ctypes.data, cev.ctypes.data, ccap)
            if rc == E_CAPACITY:
                need_p = int(offs[-1])
                need_c = int(coffs[-1]) if children and need_p <= pcap else ccap
                pcap, ccap = max(pcap, need_p), max(ccap, need_c)
                continue
            _check(rc)
            p, t = int(offs[-1]), int(coffs[int(offs[-1])]) if children else 0
            return offs, status, pos[:p], coffs[:p + 1], cmv[:t], cev[:t], (pcap, ccap)
        raise GnError(E_CAPACITY, "capacity retry failed")

    def host_stages(self):
        """Stage times (ms) of the last gn_evaluate_games / gn_expand_and_evaluate (GN_STAT_HOST_*)."""
        return {k: self.get_option(v) / 1e6 for k, v in HOST_STAGES.items()}

    def perft(self, fen: str, depth: int) -> int:
        v = C.c_uint64()
        _check(lib().gn_perft(self.h, fen.encode(), depth, C.byref(v)))
        return v.value

    # ---- device-resident API -------------------------------------------
    def alloc(self, nbytes, slot=0) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes, slot)

    def evaluate_device(self, d_boards: DeviceBuffer, n, mode, d_out: DeviceBuffer, stream=None, slot=0):
        _check(lib().gn_evaluate_device(self.h, slot, d_boards.ptr, n, mode, d_out.ptr, stream))

    def random_positions_device(self, seed, first, n, max_plies, d_out: DeviceBuffer, stream=None, slot=0):
        _check(lib().gn_random_positions_device(self.h, slot, seed, first, n, max_plies, d_out.ptr, stream))

    def set_option(self, option, value):
        _check(lib().gn_set_option(self.h, option, value))

    def get_option(self, option):
        v = C.c_int64()
        _check(lib().gn_get_option(self.h, option, C.byref(v)))
        return v.value

    def random_games_device(self, seed, first_game, n_games, plies, d_out: DeviceBuffer, stream=None, slot=0):
        _check(lib().gn_random_games_device(self.h, slot, seed, first_game, n_games, plies, d_out.ptr, stream))

    def time_expand_device(self, d_parents: DeviceBuffer, n, mode, iters, slot=0, outputs=None):
        """outputs: optional dict of DeviceBuffers po (parents), off (u32 offsets), mv (moves), co (children)
        plus cap; they receive the timed expansion's results."""
        ms, total, rows = C.c_float(), C.c_size_t(), C.c_uint64()
        st = (C.c_float * len(EXPAND_STAGES))()
        o = outputs or {}
        ptr = lambda k: o[k].ptr if k in o else None
        _check(lib().gn_time_expand_device(self.h, slot, d_parents.ptr, n, mode, iters, C.byref(ms),
                                           C.byref(total), st, C.byref(rows), ptr("po"), ptr("off"), ptr("mv"),
                                           ptr("co"), o.get("cap", 0)))
        return ms.value, total.value, list(st), rows.value

    def checksum_device(self, d_buf: DeviceBuffer, nbytes=None, offset=0, slot=0):
        """gn_checksum_device over nbytes of d_buf starting at byte offset."""
        v = C.c_uint64()
        _check(lib().gn_checksum_device(self.h, slot, C.c_void_p(d_buf.addr + offset),
                                        d_buf.nbytes - offset if nbytes is None else nbytes, C.byref(v)))
        return v.value

    def synchronize(self, slot=0):
        _check(lib().gn_synchronize(self.h, slot))

    def time_evaluate_device(self, d_boards, n, mode, d_out, iters, per_kernel=True, slot=0, rows=False):
        ms, r = C.c_float(), C.c_uint64()
        pk = (C.c_float * 4)() if per_kernel else None
        _check(lib().gn_time_evaluate_device(self.h, slot, d_boards.ptr, n, mode, d_out.ptr, iters,
                                             C.byref(ms), pk, C.byref(r) if rows else None))
        out = (ms.value, (list(pk) if per_kernel else None))
        return out + (r.value,) if rows else out

    def expand_device(self, d_parents, n, mode, d_parent_out, d_offsets, d_children, d_moves, d_child_out,
                      cap, stream=None, slot=0):
        total = C.c_size_t()
        _check(lib().gn_expand_device(self.h, slot, d_parents.ptr, n, mode,
                                      d_parent_out.ptr if d_parent_out else None, d_offsets.ptr,
                                      d_children.ptr, d_moves.ptr, d_child_out.ptr, cap, C.byref(total),
                                      stream))
        return total.value

    def expand2_device(self, d_parents, n, mode, out, stream=None, slot=0):
        """Depth 2 (gn_expand2_device).  out: DeviceBuffers po, off, ch (child boards), mv, co,
        goff, gmv, gco, plus caps cap / gcap.  Returns (children, grandchildren); with
        E_CAPACITY the counts needed are in the exception's .need."""
        t, g = C.c_size_t(), C.c_size_t()
        p = lambda k: out[k].ptr if out.get(k) is not None else None
        rc = lib().gn_expand2_device(self.h, slot, d_parents.ptr, n, mode, p("po"), p("off"), p("ch"), p("mv"),
                                     p("co"), out.get("cap", 0), p("goff"), p("gmv"), p("gco"), out.get("gcap", 0),
                                     C.byref(t), C.byref(g), stream)
        if rc == E_CAPACITY:
            e = GnError(rc, (lib().gn_last_error() or b"").decode(errors="replace"))
            e.need = (t.value, g.value)
            raise e
        _check(rc)
        return t.value, g.value


def move_to_uci(m: int) -> str:
    """Stockfish move encoding -> UCI text (castling as king-takes-rook, Chess960 style)."""
    to, frm, typ = m & 63, (m >> 6) & 63, m >> 14
    sq = lambda s: "abcdefgh"[s & 7] + str((s >> 3) + 1)
    return sq(frm) + sq(to) + ("nbrq"[(m >> 12) & 3] if typ == 1 else "")
