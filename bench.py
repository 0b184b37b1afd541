#!/usr/bin/env python3
"""bench.py — batched Stockfish NNUE evaluation throughput on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, N>1 under
`torch.distributed.run`; rank 0 prints ONE JSON line.  Run without a launcher
(WORLD_SIZE unset) with --gpus N > 1, bench.py starts the N ranks itself: it runs
`torch.distributed.run` as a child process before anything touches the GPU and exits
with its code.  Under a launcher, WORLD_SIZE must equal --gpus (else exit code 2).

Default workload `expand` (BASELINE.json configs[4], the 1/2/4/8-GPU scaling
configuration; configs[3]'s batch shape): every GPU holds 49,152 random 80-ply
games = 3,981,312 parent positions (81 per game), and one step is
  legal-child generation (GPU bitboard movegen, count + scan + write with
  per-child FT deltas) + big-net evaluation of every parent and every legal
  child (children incremental from the parent accumulators, consecutive game
  positions chained, king-move refreshes from the block's king cache) + the
  Eval::evaluate epilogue with to_cp,
~127 M evaluated positions per GPU per step, i.e. >= 1e9 per step on 8 GPUs.
The timed step's own outputs are verified: a device checksum of every parent and
child result against the same expansion run the plain way (one workgroup per
parent, every parent refreshed, no king cache), and sampled parents with all
their children against the CPU oracle.
Secondary results (same JSON object, not `value`):
  big16m  configs[2]: big-net full refresh of 16,777,216 positions per GPU;
  small1m configs[1]: small-net evaluation of 1,048,576 positions per GPU;
each with an oracle check of 4,096 of the timed outputs.

All inputs are generated on the GPU by the same seeded playout code the host
uses (`value` never includes host transfers), per-GPU work is fixed as N grows
("scaling": "weak"), and there is no data-path collective: RCCL
(torch.distributed "nccl") only broadcasts the .nnue images from rank 0 and
gathers per-rank checksums, check results and the max wall time.  Ranks shard
games by the library's partitioner (gn_partition).  Nets: GPU_NNUE_BIG /
GPU_NNUE_SMALL if set (real Stockfish nets), else seeded synthetic nets of
identical shape (fishnet_amd/synthnet.py).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NNUE evals/sec (node) at 1/2/4/8 MI355X + FT gather HBM GB/s as % of peak"
# /opt/skills/guides/MI355X_MICROARCH.md: HBM3E 8 TB/s peak; L2 34.5 TB/s aggregate (§L2);
# gathered rows past L2 (§Indexed rows: gather into LDS): 7.4-7.9 TB/s for uniformly random
# rows of a 151 MB table, the row of that table that matches the 141 MB big-net FT table
# (its top, 7.9, is the ceiling used; rounds 1-2 used the 38 MB table's 8.6)
HBM_PEAK_GBS = 8000.0
L2_PEAK_GBS = 34500.0
IC_GATHER_GBS = 7900.0
SEED = 0x5EED0000
PLIES = 80
WORKLOADS = {
    "expand": dict(mode=1, n=49152, l1=3072, config=(
        "configs[4] (configs[3] batch shape): 49,152 random 80-ply games per MI355X = 3,981,312 parents x every "
        "legal child; GPU movegen + big-net (L1=3072) evaluation, children incremental from the parent "
        "accumulators; >= 1e9 evaluated positions per step at 8 GPUs")),
    "big16m": dict(mode=1, n=1 << 24, l1=3072, config=(
        "configs[2]: big-net (L1=3072) evaluation of 16,777,216 random-playout positions per MI355X, full refresh")),
    "small1m": dict(mode=2, n=1 << 20, l1=128, config=(
        "configs[1]: small-net (L1=128) evaluation of 1,048,576 random-playout positions per MI355X")),
    "full16m": dict(mode=0, n=1 << 24, l1=3072, config=(
        "Eval::evaluate pipeline (small net, big-net re-eval when |nnue| < 236) on 16,777,216 positions per MI355X")),
}
EVAL_STAGES = ["classify_sort", "small_net", "big_net", "finalize"]


def popcounts(occ: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(occ).view(np.uint8).reshape(-1, 8)
    table = np.array([bin(i).count("1") for i in range(256)], dtype=np.uint8)
    return table[b].sum(axis=1, dtype=np.int64)


def cpuinfo():
    info = {"model": platform.processor() or "unknown", "flags": set(), "vendor": "", "family": 0}
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                info["model"] = v
            elif k == "flags":
                info["flags"] = set(v.split())
            elif k == "vendor_id":
                info["vendor"] = v
            elif k == "cpu family":
                info["family"] = int(v)
            if info["flags"] and info["vendor"] and info["family"] and k == "flags":
                break
    except OSError:
        pass
    return info


def fishnet_cpu_class(info) -> str:
    """The Stockfish build fishnet would pick on this CPU: Cpu::detect + Cpu::requirements
    (/root/reference/src/assets.rs:52-121), best first."""
    f = info["flags"]
    sse41 = "sse4_1" in f and "popcnt" in f
    avx2 = sse41 and "avx2" in f
    bmi2 = avx2 and "bmi2" in f and (info["vendor"] != "AuthenticAMD" or info["family"] >= 0x19)
    avx512 = bmi2 and "avx512f" in f and "avx512bw" in f
    vnni = avx512 and {"avx512dq", "avx512vl", "avx512_vnni"} <= f
    for ok, name in ((vnni, "x86-64-vnni256"), (avx512, "x86-64-avx512"), (bmi2, "x86-64-bmi2"),
                     (avx2, "x86-64-avx2"), (sse41, "x86-64-sse41-popcnt")):
        if ok:
            return name
    return "x86-64"


def host_threads():
    """This GPU's share of host cores: the affinity mask, capped by OMP_NUM_THREADS (the
    GPU pool sets it to its per-GPU CPU share)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(aff, int(omp))) if omp.isdigit() and int(omp) > 0 else aff


def roofline(alg_bytes, kern_ms, kernel, pmc, launches=1):
    """Hierarchical memory ceiling of the FT row gather: every gathered row byte passes
    the L2 (34.5 TB/s), the bytes past L2 (PMC traffic) come from the Infinity Cache /
    HBM (8.6 TB/s for gathered rows); the kernel cannot beat the slower of the two.
    Without PMC data only the L2 term is known (frac then a lower bound)."""
    t = kern_ms * 1e-3
    achieved = alg_bytes / t / 1e9
    t_l2 = alg_bytes / (L2_PEAK_GBS * 1e9)
    r = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "unit": "GB/s",
         "traffic": None, "alg_bytes_per_launch": int(alg_bytes), "kernel_ms_per_launch": round(kern_ms, 4),
         "launches_per_step": launches,
         "peak_model": "alg_bytes / max(alg_bytes / 34.5 TB/s (L2), traffic / 7.9 TB/s (gathered rows past L2, "
                       "151 MB table row of MI355X_MICROARCH.md)); achieved = kernel-counted FT rows x "
                       "(2*L1/S + 4) B (the launch's S-th of the row + its 4-B list entry; S = launches_per_step "
                       "column slices) / the launch's time"}
    if pmc:
        traffic = float(pmc["hbm_side_bytes_per_launch"])
        t_ic = traffic / (IC_GATHER_GBS * 1e9)
        peak = alg_bytes / max(t_l2, t_ic) / 1e9
        r.update(traffic=int(traffic), traffic_source=pmc["source"], l2_hit_rate=pmc.get("l2_hit_rate"),
                 hbm_side_GBps=round(traffic / t / 1e9, 1), hbm_frac=round(traffic / t / 1e9 / HBM_PEAK_GBS, 4))
    else:
        peak = L2_PEAK_GBS
    r["peak"] = round(peak, 1)
    r["frac"] = round(achieved / peak, 4)
    return r


class Ctx:
    """Per-rank state: library context + the RCCL plumbing of fishnet_amd/dist.py (comm: an
    object with ShardComm's interface; default ShardComm("nccl"), one rank per GPU)."""

    def __init__(self, args, comm=None):
        import torch  # first: torch's HIP runtime is then the one libgpu_nnue binds to
        from fishnet_amd.dist import ShardComm
        self.torch = torch
        self.comm = comm if comm is not None else ShardComm("nccl")
        self.rank, self.world, self.local = self.comm.rank, self.comm.world, self.comm.local
        from fishnet_amd import build, gpu_nnue as G, synthnet
        if not os.environ.get("GPU_NNUE_LIB"):  # (an A/B variant library is built beforehand)
            build.build()
        self.G = G
        # nets: rank 0 reads, RCCL broadcast over xGMI, every rank loads from memory
        big_p, small_p, label = synthnet.net_paths() if self.rank == 0 else (None, None, None)
        blobs = [self.comm.broadcast_bytes(open(p, "rb").read() if self.rank == 0 else b"") for p in (big_p, small_p)]
        self.blobs = blobs
        self.net_label = self.comm.broadcast_obj(label)
        self.nn = G.GpuNnue(big_bytes=blobs[0], small_bytes=blobs[1], devices=[self.local])
        if args.swizzle >= 0:
            self.nn.set_option(G.OPT_XCD_SWIZZLE, args.swizzle)
        if args.king_sort >= 0:
            self.nn.set_option(G.OPT_KING_SORT, args.king_sort)
        if args.chain is not None:
            self.nn.set_option(G.OPT_CHAIN, args.chain)
        if args.king_cache is not None:
            self.nn.set_option(G.OPT_KING_CACHE, args.king_cache)
        if getattr(args, "pipeline", None) is not None:
            self.nn.set_option(G.OPT_EXPAND_PIPELINE, args.pipeline)
        self.options = {"xcd_swizzle": self.nn.get_option(G.OPT_XCD_SWIZZLE),
                        "king_sort": self.nn.get_option(G.OPT_KING_SORT),
                        "incremental_children": self.nn.get_option(G.OPT_INCREMENTAL_CHILDREN),
                        "chain": self.nn.get_option(G.OPT_CHAIN), "king_cache": self.nn.get_option(G.OPT_KING_CACHE),
                        "expand_pipeline": self.nn.get_option(G.OPT_EXPAND_PIPELINE)}
        self._onets = None

    def oracle_nets(self):
        """(oracle module, big net, small net) from the broadcast images (rank-local CPU)."""
        if self._onets is None:
            from oracle import oracle as O
            O.build()
            self._onets = (O, O.Net(data=self.blobs[0]), O.Net(data=self.blobs[1]))
        return self._onets

    def shard(self, items_per_rank):
        """(first, count) of this rank's items by the library's partitioner (equal weights)."""
        b = self.G.partition(items_per_rank * self.world, self.world)
        return b[self.rank], b[self.rank + 1] - b[self.rank]

    def barrier_sync(self):
        self.comm.barrier()
        self.torch.cuda.synchronize()

    def close(self):
        self.comm.close()
        self.nn.close()


def run_eval(c: Ctx, wl: dict, n: int, steps: int, warmup: int, max_plies: int, check: int):
    """Full-refresh batch evaluation of n device-resident positions per GPU."""
    G, nn, mode = c.G, c.nn, wl["mode"]
    d_b, d_o = nn.alloc(n * 32), nn.alloc(n * G.EVAL_SIZE)
    t = time.perf_counter()
    first, _ = c.shard(n)
    nn.random_positions_device(SEED, first, n, max_plies, d_b)
    nn.synchronize()
    gen_s = time.perf_counter() - t
    for _ in range(warmup):
        nn.evaluate_device(d_b, n, mode, d_o)
    nn.synchronize()
    c.barrier_sync()
    t0 = time.perf_counter()
    _, stage, rows = nn.time_evaluate_device(d_b, n, mode, d_o, steps, per_kernel=True, rows=True)
    c.barrier_sync()
    wall = c.comm.max(time.perf_counter() - t0)
    out, boards = d_o.download(G.EVAL_DTYPE, n), d_b.download(G.BOARD_DTYPE, n)
    checksum = nn.checksum_device(d_o, n * G.EVAL_SIZE)
    d_b.free(), d_o.free()
    pieces = popcounts(boards["occ"])
    alg = rows * (2 * wl["l1"] + 4) + n * 40
    k = 1 if mode == 2 else 2
    r = dict(value=c.world * n * steps / wall, wall=wall, stage=stage, kern_ms=stage[k], alg=alg, rows=rows, out=out,
             boards=boards, pieces=pieces, gen_s=gen_s, checksum=checksum,
             kernel=f"eval_net<{wl['l1']}> ({EVAL_STAGES[k]})")
    if check:  # the timed launch's own outputs, first `check` positions, against the oracle
        O, big, small = c.oracle_nets()
        k = min(check, n)
        fens = [G.board_to_fen(b) for b in boards[:k]]
        exp = O.eval_fens(big if mode != 2 else None, small if mode != 1 else None, fens, mode,
                          threads=host_threads())
        r["oracle_check"] = {"positions": k, "mismatches": int(np.count_nonzero(exp != out[:k])),
                             "of": "the timed launch's outputs"}
    return r


def run_expand(c: Ctx, wl: dict, games: int, steps: int, warmup: int, check: int, gather: bool | None = None):
    """Games x 81 parents, every legal child, incremental evaluation; verifies the timed outputs."""
    G, nn, mode = c.G, c.nn, wl["mode"]
    n = games * (PLIES + 1)
    d_p = nn.alloc(n * 32)
    t = time.perf_counter()
    first, _ = c.shard(games)
    nn.random_games_device(SEED, first, games, PLIES, d_p)
    nn.synchronize()
    gen_s = time.perf_counter() - t
    # one untimed expansion sizes the output buffers (and warms up); then W warmup steps.  The
    # outputs live in torch tensors (device memory the library writes through raw pointers), so
    # that RCCL can gather them at N > 1
    _, total, _, _ = nn.time_expand_device(d_p, n, mode, 1)
    tb = lambda nb: G.DeviceView(nn, c.torch.empty(max(nb, 1), dtype=c.torch.uint8, device=c.comm.device))
    out = {"po": tb(n * G.EVAL_SIZE), "off": tb((n + 1) * 4), "mv": tb(max(total, 1) * 2),
           "co": tb(max(total, 1) * G.EVAL_SIZE), "cap": total}
    if warmup:
        nn.time_expand_device(d_p, n, mode, warmup, outputs=out)
    c.barrier_sync()
    t0 = time.perf_counter()
    _, children, stage, rows = nn.time_expand_device(d_p, n, mode, steps, outputs=out)
    c.barrier_sync()
    wall = c.comm.max(time.perf_counter() - t0)
    scratch_pads = nn.get_option(G.STAT_SCRATCH_PADS)
    # the big net's two kernels timed apart (HIP events on the library's stream, inside the
    # timed region): the roofline's dominant kernel is stream_eval_kernel alone
    plan_ms, stream_ms = nn.get_option(G.STAT_PLAN_NS) / 1e6, nn.get_option(G.STAT_STREAM_NS) / 1e6
    finish_ms = nn.get_option(G.STAT_FINISH_NS) / 1e6  # the sliced stream's slice_finish_kernel
    parents = d_p.download(G.BOARD_DTYPE, n)
    sums = (nn.checksum_device(out["po"], n * G.EVAL_SIZE), nn.checksum_device(out["co"], children * G.EVAL_SIZE),
            nn.checksum_device(out["mv"], children * 2), nn.checksum_device(out["off"], (n + 1) * 4))
    planned = stream_ms > 0
    # the column-sliced stream (GN_OPT_STREAM_SLICES 3): three launches per step, each over a
    # third of every row's columns; the roofline is per launch (= rocprofv3's per-dispatch view)
    sl = 3 if planned and wl["l1"] == 3072 and nn.get_option(G.OPT_STREAM_SLICES) == 3 else 1
    r = dict(value=c.world * (n + children) * steps / wall, wall=wall, stage=stage,
             kern_ms=(stream_ms / sl) if planned else stage[5 if mode != 2 else 4], plan_ms=plan_ms,
             finish_ms=finish_ms,
             alg=rows * (2 * wl["l1"] // sl + 4), rows=rows, parents=parents, n=n, launches=sl,
             children=children, gen_s=gen_s, checksum=sums[0] ^ sums[1], scratch_pads=scratch_pads,
             kernel=(f"stream_eval_kernel<{wl['l1']}, 3> (3 column-slice launches per step)" if sl == 3 else
                     f"stream_eval_kernel<{wl['l1']}>") if wl["l1"] != 128 else f"expand_eval<{wl['l1']}>")
    if check:
        ver = {}
        # (1) sampled parents of the timed outputs, with all their children, against the oracle
        O, big, small = c.oracle_nets()
        rng = np.random.default_rng(1234 + c.rank)
        idx = np.unique(np.concatenate([rng.choice(n, size=min(check, n), replace=False),
                                        np.arange(min(81, n))]))  # + one whole game (its chain and king cache)
        offs = out["off"].download(np.uint32, n + 1)
        fens = [G.board_to_fen(parents[i]) for i in idx]
        pev = out["po"].download(G.EVAL_DTYPE, n)

        def one(j):
            i = int(idx[j])
            lo, hi = int(offs[i]), int(offs[i + 1])
            mv = out["mv"].download(np.uint16, hi - lo, offset=lo)
            ev = out["co"].download(G.EVAL_DTYPE, hi - lo, offset=lo)
            p_exp, m_exp, k_exp = O.expand_eval(big if mode != 2 else None, small if mode != 1 else None, fens[j],
                                                mode, incremental=True)
            got = dict(zip(mv.tolist(), map(tuple, ev.tolist())))
            return int(got != dict(zip(m_exp, map(tuple, k_exp.tolist()))) or tuple(pev[i]) != p_exp), hi - lo

        with cf.ThreadPoolExecutor(host_threads()) as ex:
            res = list(ex.map(one, range(len(idx))))
        ver["oracle"] = {"parents": len(idx), "children": sum(x[1] for x in res),
                         "mismatching_parents": sum(x[0] for x in res),
                         "of": "the timed expansion's outputs (random parents + the first whole game)"}
        # (2) every output of the timed step against the plain path: one workgroup per parent,
        # every parent refreshed, no king cache (GN_OPT_CHAIN 1, GN_OPT_KING_CACHE 0)
        opts = (nn.get_option(G.OPT_CHAIN), nn.get_option(G.OPT_KING_CACHE))
        try:
            nn.set_option(G.OPT_CHAIN, 1)
            nn.set_option(G.OPT_KING_CACHE, 0)
            _, t2, _, _ = nn.time_expand_device(d_p, n, mode, 1, outputs=out)
        finally:
            nn.set_option(G.OPT_CHAIN, opts[0])
            nn.set_option(G.OPT_KING_CACHE, opts[1])
        ref = (nn.checksum_device(out["po"], n * G.EVAL_SIZE), nn.checksum_device(out["co"], t2 * G.EVAL_SIZE),
               nn.checksum_device(out["mv"], t2 * 2), nn.checksum_device(out["off"], (n + 1) * 4))
        ver["vs_plain_path"] = {"equal": bool(ref == sums and t2 == children), "parents": n, "children": children,
                                "checksum_timed": f"{sums[0] ^ sums[1]:016x}",
                                "checksum_plain": f"{ref[0] ^ ref[1]:016x}",
                                "plain_path": "GN_OPT_CHAIN=1, GN_OPT_KING_CACHE=0 (refresh-started parents)"}
        r["oracle_check"] = ver
    if c.world > 1 if gather is None else gather:  # (gather=True: also at N = 1, tests)
        r["gather"] = gather_results(c, out, n, children, games, mode, check)
    for b in ("po", "off", "mv", "co"):
        out[b].free()
    out.clear()
    d_p.free()
    return r


def gather_records(c, out, n, children):
    """Every rank's records of one expansion to rank 0 (ShardComm.gather_tensor: RCCL on device
    tensors, gloo on CPU tensors; the lengths differ per rank): parent gn_eval records, the child
    offsets, child moves and child gn_eval records.  Returns ({part: list of every rank's bytes
    on rank 0, None elsewhere}, bytes of all ranks)."""
    es = c.G.EVAL_SIZE
    parts = (("po", n * es), ("off", (n + 1) * 4), ("mv", children * 2), ("co", children * es))
    got = {k: c.comm.gather_tensor(out[k].tensor[:nb]) for k, nb in parts}
    if out["po"].tensor.is_cuda:
        c.torch.cuda.synchronize()
    return got, sum(c.comm.gather_i64(sum(nb for _, nb in parts)))


def gather_results(c: Ctx, out, n, children, games, mode, check):
    """The result gather of DESIGN.md section 6 (N > 1): every rank's parent / child records, child
    moves and offsets of the timed step to rank 0 over RCCL (torch.distributed gather on the
    records' device memory), outside the timed region and timed on its own; rank 0 then checks
    sampled parents of every rank, with all their children, against the oracle."""
    G = c.G
    es = G.EVAL_SIZE
    c.barrier_sync()
    t0 = time.perf_counter()
    got, nbytes = gather_records(c, out, n, children)
    c.barrier_sync()
    ms = c.comm.max(time.perf_counter() - t0) * 1e3
    r = {"bytes_all_ranks": nbytes, "ms": round(ms, 2), "GBps_into_rank0": round(nbytes / ms / 1e6, 1),
         "how": "torch.distributed.gather (RCCL over xGMI) of each rank's gn_eval records, child moves and offsets "
                "to rank 0's device memory, after the timed steps"}
    bad = 0
    if c.rank == 0 and check:
        O, big, small = c.oracle_nets()
        bounds = G.partition(games * c.world, c.world)
        d_b = c.nn.alloc(n * 32)
        rng = np.random.default_rng(4321)
        checked = 0
        for rr in range(c.world):
            c.nn.random_games_device(SEED, bounds[rr], games, PLIES, d_b)
            c.nn.synchronize()
            boards = d_b.download(G.BOARD_DTYPE, n)
            po = got["po"][rr].cpu().numpy().view(G.EVAL_DTYPE)
            off = got["off"][rr].cpu().numpy().view(np.uint32)
            for i in rng.choice(n, size=min(32, n), replace=False):
                lo, hi = int(off[i]), int(off[i + 1])
                mv = got["mv"][rr][2 * lo:2 * hi].cpu().numpy().view(np.uint16)
                ev = got["co"][rr][es * lo:es * hi].cpu().numpy().view(G.EVAL_DTYPE)
                p_exp, m_exp, k_exp = O.expand_eval(big if mode != 2 else None, small if mode != 1 else None,
                                                    G.board_to_fen(boards[i]), mode, incremental=True)
                bad += int(tuple(po[i]) != p_exp or dict(zip(mv.tolist(), map(tuple, ev.tolist()))) !=
                           dict(zip(m_exp, map(tuple, k_exp.tolist()))))
                checked += 1
        d_b.free()
        r["oracle_check"] = {"parents": checked, "ranks": c.world, "mismatching_parents": bad,
                             "of": "the gathered records on rank 0"}
    del got
    return r


def run_expand2(c: Ctx, games: int, mode: int, steps: int, check: int):
    """Depth 2 (gn_expand2_device): games x 81 parents, every legal child, and every legal
    child of every child, each level incremental from its parent's accumulators."""
    G, nn = c.G, c.nn
    n = games * (PLIES + 1)
    d_p = nn.alloc(n * 32)
    first, _ = c.shard(games)
    nn.random_games_device(SEED + 2, first, games, PLIES, d_p)
    nn.synchronize()
    out = {"po": nn.alloc(n * G.EVAL_SIZE), "off": nn.alloc((n + 1) * 4), "cap": 0, "gcap": 0}
    for _ in range(3):  # sized by the library's own capacity replies (also the warmup)
        try:
            t, g = nn.expand2_device(d_p, n, mode, out)
            break
        except G.GnError as e:
            if e.code != G.E_CAPACITY:
                raise
            t, g = e.need
            if t > out["cap"]:
                out.update(cap=t, ch=nn.alloc(t * 32), mv=nn.alloc(t * 2), co=nn.alloc(t * G.EVAL_SIZE), goff=nn.alloc((t + 1) * 4))
            if g > out["gcap"]:
                out.update(gcap=g, gmv=nn.alloc(max(g, 1) * 2), gco=nn.alloc(max(g, 1) * G.EVAL_SIZE))
    c.barrier_sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        t, g = nn.expand2_device(d_p, n, mode, out)
    c.barrier_sync()
    wall = c.comm.max(time.perf_counter() - t0)
    r = {"workload": f"depth 2: {games} random 80-ply games per MI355X = {n} parents, their {t} legal children and "
                     f"{g} grandchildren (gn_expand2_device, big net, every level incremental)",
         "value": round(c.world * (n + t + g) * steps / wall, 1), "unit": "evals/s",
         "ms_per_step": round(wall * 1e3 / steps, 3), "children": t, "grandchildren": g}
    if check:  # the timed call's own outputs: sampled children's grandchildren vs the oracle
        O, big, small = c.oracle_nets()
        rng = np.random.default_rng(99 + c.rank)
        idx = np.unique(rng.choice(t, size=min(check, t), replace=False))
        kids = out["ch"].download(G.BOARD_DTYPE, t)
        co = out["co"].download(G.EVAL_DTYPE, t)
        goff = out["goff"].download(np.uint32, t + 1)
        fens = [G.board_to_fen(kids[j]) for j in idx]

        def one(k):
            j = int(idx[k])
            lo, hi = int(goff[j]), int(goff[j + 1])
            mv = out["gmv"].download(np.uint16, hi - lo, offset=lo)
            ev = out["gco"].download(G.EVAL_DTYPE, hi - lo, offset=lo)
            p_exp, m_exp, k_exp = O.expand_eval(big, small, fens[k], mode, incremental=True)
            # (co[j] is a child record, p_exp the same position scored: compare the static part)
            static = lambda t: tuple(t)[:4] + (int(tuple(t)[5]) & 15,)
            return int(static(co[j]) != static(p_exp) or dict(zip(mv.tolist(), map(tuple, ev.tolist()))) !=
                       dict(zip(m_exp, map(tuple, k_exp.tolist())))), hi - lo

        with cf.ThreadPoolExecutor(host_threads()) as ex:
            res = list(ex.map(one, range(len(idx))))
        r["oracle_check"] = {"children": len(idx), "grandchildren": sum(x[1] for x in res),
                             "mismatching_children": sum(x[0] for x in res),
                             "of": "the timed call's outputs (random children with all their children)"}
    for b in out.values():
        if hasattr(b, "free"):
            b.free()
    d_p.free()
    return r


START_FEN = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def run_abi_games(c: Ctx, games: int, mode: int, steps: int, check: int):
    """secondary.abi_games: the C-ABI's host-facing path as fishnet would call it.  Lichess-shaped
    batches (root FEN + the game's UCI moves as one string, AcquireResponseBody) in host memory ->
    gn_evaluate_games(with_children=1) -> every position's and every legal child's record in host
    memory (the caller's reused numpy arrays).  Inside the call: host FEN parse + move
    tokenizing, upload, the GPU replay of the moves, the expansion in chunks of whole games, the
    downloads overlapped with the next chunk.  Verified: sampled positions with all children vs
    the oracle, and the first full-length games vs the device-resident expansion of the same
    games (gn_random_games_device + gn_expand_device)."""
    G, nn = c.G, c.nn
    first, _ = c.shard(games)
    seed = SEED + 3
    t = time.perf_counter()
    ucis = G.random_games_uci(seed, first, games, PLIES)
    arr, keep = G._games_array([(START_FEN, u, ()) for u in ucis])
    prep_s = time.perf_counter() - t
    bufs = {}
    res = nn.evaluate_games_arrays(arr, games, mode, True, bufs=bufs)  # sizes the buffers (and warms up)
    caps = res[-1]
    c.barrier_sync()
    t0 = time.perf_counter()
    stages, calls = [], []
    for _ in range(steps):
        t1 = time.perf_counter()
        res = nn.evaluate_games_arrays(arr, games, mode, True, caps, bufs)
        calls.append(time.perf_counter() - t1)
        stages.append(nn.host_stages())
    c.barrier_sync()
    wall = c.comm.max(time.perf_counter() - t0)
    offs, status, pos, coffs, cmv, cev, _ = res
    npos, nch = len(pos), len(cev)
    st = {k: round(sum(s[k] for s in stages) / len(stages), 3) for k in stages[0]}
    r = {"workload": f"C-ABI host path: {games} lichess-shaped games per MI355X (start position + {PLIES} random plies "
                     f"as one UCI string each, AcquireResponseBody form) -> gn_evaluate_games(with_children=1): "
                     f"{npos} positions + {nch} legal children, records in host memory",
         "value": round(c.world * (npos + nch) * steps / wall, 1), "unit": "evals/s",
         "ms_per_call": round(wall * 1e3 / steps, 3), "positions": npos, "children": nch,
         "result_bytes_to_host": int(npos * G.EVAL_SIZE + nch * (G.CHILD_SIZE + 2) + (npos + 1) * 4),
         "records": "positions: 24-B gn_eval (with the score); children: 12-B gn_child (ABI v4) + 2-B move",
         "stage_ms": st, "python_call_ms": round(1e3 * sum(calls) / len(calls), 3), "prep_s_untimed": round(prep_s, 2),
         "stages": "parse: host root FEN + UCI tokenizing; upload: inputs to the device; replay: the GPU replay of "
                   "the moves; compute: children + evaluation + score rule over all chunks (main thread); "
                   "download: device->host record copies, all chunks (a drain thread, overlapping the next "
                   "chunk); tail: downloads left after the last chunk computed; total: the call"}
    if check:
        O, big, small = c.oracle_nets()
        rng = np.random.default_rng(77 + c.rank)
        ok = np.nonzero(status[:games] == 0)[0]
        gi = rng.choice(ok, size=min(check, len(ok)), replace=False)
        items = [(int(g), int(rng.integers(0, int(offs[g + 1] - offs[g])))) for g in gi]

        def one(it):
            g, k = it
            fens, _ = O.replay_game(START_FEN, ucis[g].split()[:k])
            at = int(offs[g]) + k
            a, b = int(coffs[at]), int(coffs[at + 1])
            p_exp, m_exp, k_exp = O.expand_eval(big if mode != 2 else None, small if mode != 1 else None, fens[-1],
                                                mode, incremental=True)
            got = dict(zip(cmv[a:b].tolist(), map(tuple, G.decode_children(cev[a:b]).tolist())))
            exp = dict(zip(m_exp, map(tuple, G.children_from_evals(k_exp).tolist())))
            return int(tuple(pos[at]) != p_exp or got != exp), b - a

        with cf.ThreadPoolExecutor(host_threads()) as ex:
            out = list(ex.map(one, items))
        ver = {"oracle": {"positions": len(items), "children": sum(x[1] for x in out),
                          "mismatching_positions": sum(x[0] for x in out)}}
        # the first full-length games against the device-resident expansion of the same games
        ng = min(512, games)
        d_b = nn.alloc(ng * (PLIES + 1) * 32)
        nn.random_games_device(seed, first, ng, PLIES, d_b)
        nn.synchronize()
        dev = d_b.download(G.BOARD_DTYPE, ng * (PLIES + 1)).reshape(ng, PLIES + 1)
        full = [g for g in range(ng) if status[g] == 0 and offs[g + 1] - offs[g] == PLIES + 1]
        sel = np.concatenate([dev[g] for g in full])
        m, cap = len(sel), int(coffs[int(offs[full[-1] + 1])] - coffs[int(offs[full[0]])]) + 1
        cap = max(cap, 64 * m)
        db = {k: nn.alloc(sz) for k, sz in (("b", m * 32), ("po", m * G.EVAL_SIZE), ("off", (m + 1) * 4),
                                               ("ch", cap * 32), ("mv", cap * 2), ("co", cap * G.EVAL_SIZE))}
        db["b"].upload(sel)
        tt = nn.expand_device(db["b"], m, mode, db["po"], db["off"], db["ch"], db["mv"], db["co"], cap)
        po, doff = db["po"].download(G.EVAL_DTYPE, m), db["off"].download(np.uint32, m + 1)
        dmv, dco = db["mv"].download(np.uint16, tt), db["co"].download(G.EVAL_DTYPE, tt)
        bad, i = 0, 0
        for g in full:
            a0, a1 = int(offs[g]), int(offs[g + 1])
            c0, c1 = int(coffs[a0]), int(coffs[a1])
            d0, d1 = int(doff[i]), int(doff[i + a1 - a0])
            bad += int(not (np.array_equal(pos[a0:a1], po[i:i + a1 - a0]) and np.array_equal(cmv[c0:c1], dmv[d0:d1])
                            and np.array_equal(G.decode_children(cev[c0:c1]), G.children_from_evals(dco[d0:d1]))))
            i += a1 - a0
        for b in list(db.values()) + [d_b]:
            b.free()
        ver["vs_device_resident"] = {"games": len(full), "positions": m, "children": tt, "mismatching_games": bad}
        r["oracle_check"] = ver
    return r


def run_dropin(c: Ctx, games: int, threads: int, calls_per_thread: int, check: int):
    """secondary.dropin: the drop-in's real call shape.  fishnet's N workers
    each send one chunk at a time (/root/reference/src/main.rs:263-343); with the GPU backend a
    chunk is one lichess game (rust/patches/0002: whole-batch chunks), which GpuEvalStub sends as
    one gn_evaluate_batch(GN_MODE_FULL) of the game's positions (root + every ply, checks and
    mates included).  Measured: (1) one caller, call after call: per-call latency; (2) `threads`
    callers at once on one context, as the stub's spawn_blocking calls arrive from the workers:
    positions/s and per-call latency, with concurrent calls merged into one launch
    (GN_OPT_COALESCE = 1, the default) and run one after another (0).  FENs are prepared untimed
    (the caller holds them); each timed call is the C call alone."""
    import ctypes as C
    import threading
    G, nn, L = c.G, c.nn, c.G.lib()
    first, _ = c.shard(games)
    ucis = G.random_games_uci(SEED + 5, first, games, PLIES)
    calls = []
    for u in ucis:
        boards, _, _ = G.replay_game(START_FEN, u)
        fens = G.boards_to_fens(boards)
        enc = [f.encode() for f in fens]
        calls.append(((C.c_char_p * len(enc))(*enc), enc, np.zeros(len(enc), dtype=G.EVAL_DTYPE), fens))

    def call(k):
        arr, enc, out, _ = calls[k % len(calls)]
        t = time.perf_counter()
        rc = L.gn_evaluate_batch(nn.h, arr, len(enc), out.ctypes.data)
        dt = time.perf_counter() - t
        if rc:
            G._check(rc)
        return dt

    def pct(xs, q):
        return round(float(np.percentile(np.array(xs) * 1e3, q)), 4)

    for k in range(min(32, len(calls))):  # warmup (buffers sized, kernels loaded)
        call(k)
    single = [call(k) for k in range(len(calls))]
    npos = sum(len(x[1]) for x in calls)
    in_check = sum(int(np.count_nonzero(x[2]["flags"] & G.FLAG_IN_CHECK)) for x in calls)
    searched = sum(int(np.count_nonzero(x[2]["flags"] & G.FLAG_SEARCHED)) for x in calls)
    r = {"workload": f"one lichess game per call (start position + up to {PLIES} random plies = "
                     f"{npos / len(calls):.1f} positions), gn_evaluate_batch(GN_MODE_FULL) as GpuEvalStub::go_multiple "
                     f"sends it; {games} games per MI355X; {in_check} of the {npos} positions in check "
                     f"({searched} scored by the in-check rule)",
         "single_caller": {"calls": len(single), "p50_ms": pct(single, 50), "p99_ms": pct(single, 99),
                           "positions_per_s": round(npos / sum(single), 1)}}
    for mode_name, co in (("coalesced", 1), ("serial", 0)):
        nn.set_option(G.OPT_COALESCE, co)
        l0, c0 = nn.get_option(G.STAT_BATCH_LAUNCHES), nn.get_option(G.STAT_BATCH_CALLS)
        lat = [[] for _ in range(threads)]
        go = threading.Barrier(threads + 1)

        def work(t):
            go.wait()
            for i in range(calls_per_thread):
                lat[t].append(call(t * calls_per_thread + i))

        th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        go.wait()
        t0 = time.perf_counter()
        for x in th:
            x.join()
        wall = time.perf_counter() - t0
        allx = [v for l in lat for v in l]
        pos = sum(len(calls[(t * calls_per_thread + i) % len(calls)][1]) for t in range(threads)
                  for i in range(calls_per_thread))
        r[f"{threads}_callers_{mode_name}"] = {
            "calls": len(allx), "positions_per_s": round(pos / wall, 1), "calls_per_s": round(len(allx) / wall, 1),
            "p50_ms": pct(allx, 50), "p99_ms": pct(allx, 99),
            "launches": nn.get_option(G.STAT_BATCH_LAUNCHES) - l0, "calls_served": nn.get_option(G.STAT_BATCH_CALLS) - c0}
    nn.set_option(G.OPT_COALESCE, 1)
    co = r[f"{threads}_callers_coalesced"]
    co["speedup_vs_serial"] = round(co["positions_per_s"] / r[f"{threads}_callers_serial"]["positions_per_s"], 3)
    if c.world == 1:  # the same calls from native threads (tools/dropin_native.c): no interpreter lock
        r[f"{threads}_callers_native"] = run_dropin_native(c, calls, threads, calls_per_thread)
    if check:  # the last records of sampled games (every game's last call wrote them) vs the oracle
        O, big, small = c.oracle_nets()
        idx = np.random.default_rng(55 + c.rank).choice(len(calls), size=min(check, len(calls)), replace=False)
        fens = [f for k in idx for f in calls[k][3]]
        got = np.concatenate([calls[k][2] for k in idx])
        exp = O.eval_fens(big, small, fens, G.MODE_FULL, threads=host_threads())
        r["oracle_check"] = {"games": len(idx), "positions": len(fens),
                             "mismatches": int(np.count_nonzero(got != exp)), "of": "the concurrent calls' records"}
    return r


def run_dropin_native(c: Ctx, calls, threads: int, calls_per_thread: int):
    """secondary.dropin's 16 callers as native threads: fishnet's workers call the C-ABI from Rust
    with no interpreter lock between them, while the Python threads above hold the GIL around every
    ctypes call.  tools/dropin_native.c (built by fishnet_amd/build.py) loads the same nets into its
    own context on this GPU, checks every call's records against a single-threaded pass of the same
    game, and times `threads` x `calls_per_thread` calls after a barrier (coalescing on)."""
    import subprocess
    import tempfile
    from fishnet_amd import build, synthnet
    exe = build.DROPIN_NATIVE
    if not os.path.exists(exe):
        return {"skipped": "tools/dropin_native.c not built (fishnet_amd/build.py build_dropin_native)"}
    big_p, small_p, _ = synthnet.net_paths()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for x in calls:
            f.write("|".join(x[3]) + "\n")
        path = f.name
    try:
        p = subprocess.run([exe, big_p, small_p, path, str(threads), str(calls_per_thread), "1"], capture_output=True,
                           text=True, timeout=180)
    finally:
        os.unlink(path)
    if p.returncode:
        raise RuntimeError(f"dropin_native failed ({p.returncode}): {p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


def cpu_baseline_eval(c: Ctx, boards, mode, budget_s):
    """The oracle built -O3 -march=native on this GPU's share of host cores, full refresh per
    position (a batch of unrelated FENs has no parent to update from)."""
    O, big, small = c.oracle_nets()
    O.build(native=True)
    O.use_library(O.NATIVE_LIB_PATH)
    try:
        th, info = host_threads(), cpuinfo()
        fens = c.G.boards_to_fens(boards)
        done, reps, t = 0, 0, time.perf_counter()
        while True:
            O.eval_fens(big if mode != 2 else None, small if mode != 1 else None, fens, mode, threads=th)
            done, reps = done + len(fens), reps + 1
            dt = time.perf_counter() - t
            if dt >= budget_s or reps >= 200:
                break
    finally:
        O.use_library(os.path.join(O.HERE, "_build", "liboracle.so"))
    return {"value": round(done / dt, 1), "unit": "evals/s", "cores": th, "kind": "port",
            "sample": f"{len(fens)} positions of rank 0's batch x {reps} passes = {done} evals in {dt:.1f} s; "
                      f"oracle/oracle.c -O3 -march=native (fishnet's Cpu::detect class on this host: "
                      f"{fishnet_cpu_class(info)}), full refresh per position, {th} threads = this GPU's share "
                      f"of the host ({os.cpu_count()} logical CPUs), {info['model']}"}


def cpu_baseline_expand(c: Ctx, parents, mode, budget_s):
    """The oracle built -O3 -march=native on this GPU's share of host cores: every parent + all
    its legal children, children updated incrementally from the parent's accumulators."""
    O, big, small = c.oracle_nets()
    O.build(native=True)
    O.use_library(O.NATIVE_LIB_PATH)
    try:
        th, info = host_threads(), cpuinfo()
        fens = c.G.boards_to_fens(parents)  # the oracle's input form, prepared untimed
        done, k, chunk, t = 0, 0, max(64, 16 * th), time.perf_counter()
        while True:  # passes over the sample until the budget is spent
            _, counts, _ = O.expand_eval_batch(big if mode != 2 else None, small if mode != 1 else None,
                                               fens[k % len(fens):k % len(fens) + chunk], mode, incremental=True,
                                               threads=th)
            done += len(counts) + int(counts[counts > 0].sum())
            k += len(counts)
            if time.perf_counter() - t >= budget_s:
                break
        dt = time.perf_counter() - t
    finally:
        O.use_library(os.path.join(O.HERE, "_build", "liboracle.so"))
    return {"value": round(done / dt, 1), "unit": "evals/s", "cores": th, "kind": "port",
            "sample": f"{done} evals ({k} parents of rank 0's games, {len(fens)} distinct, + all their legal children) "
                      f"in {dt:.1f} s; "
                      f"oracle/oracle.c -O3 -march=native (fishnet's Cpu::detect class on this host: "
                      f"{fishnet_cpu_class(info)}), children incremental from the parent accumulators, "
                      f"{th} threads = this GPU's share of the host ({os.cpu_count()} logical CPUs), {info['model']}"}


def load_pmc(workload, n, launches=1):
    """The last profile round's PMC figures of this workload's dominant kernel, when they were
    taken on the same shape (positions, ABI, launches per step: 3 for the column-sliced stream)."""
    p = os.path.join(ROOT, "profiles", "latest_pmc.json")
    if not os.path.exists(p):
        return None
    e = json.load(open(p)).get(workload)
    ok = e and e.get("positions") == n and e.get("abi", 1) >= 3 and e.get("launches_per_step", 1) == launches
    return e if ok else None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(gpus: int, argv) -> int | None:
    """The N > 1 launch (the reference's analog is the per-core worker fan-out,
    /root/reference/src/main.rs:151-161): with WORLD_SIZE unset and gpus > 1, run
    `torch.distributed.run` with one rank per GPU over 127.0.0.1 as a CHILD process (this process
    has not touched the GPU: no torch / HIP import yet) and return its exit code.  Under a
    launcher (WORLD_SIZE set) the world must equal gpus: a mismatch returns 2 before any GPU
    work.  None: run this process as the (only) rank."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}: launch one rank per GPU "
                  f"(torch.distributed.run --nproc-per-node {gpus})", file=sys.stderr, flush=True)
            return 2
        return None
    if gpus <= 1:
        return None
    # build the HIP library and the oracle once, here, before any rank exists (hipcc and gcc need
    # no GPU): N ranks finding a stale build would otherwise compile the same files at once
    # (--launch-check: no GPU work and no library, so the CPU launcher test needs no ROCm toolchain)
    if "--launch-check" not in argv:
        if not os.environ.get("GPU_NNUE_LIB"):
            from fishnet_amd import build
            build.build()
        from oracle import oracle as O
        O.build()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def launch_check() -> int:
    """--launch-check: no GPU work; every rank joins a gloo group and rank 0 prints the ranks it
    sees (tests/test_dist.py drives the launcher this way on the CPU)."""
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    ranks = [rank]
    if world > 1:
        dist.init_process_group("gloo")
        lst = [None] * world
        dist.all_gather_object(lst, (rank, int(os.environ.get("LOCAL_RANK", "0"))))
        ranks = lst
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "ranks": ranks}), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="expand")
    ap.add_argument("--positions", type=int, default=0, help="positions (or games for expand) per GPU")
    ap.add_argument("--max-plies", type=int, default=160)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--check", type=int, default=256,
                    help="expand: parents (with children) of the timed outputs re-checked against the oracle, plus "
                         "the plain-path checksum; eval: positions (x16, >= 4096)")
    ap.add_argument("--swizzle", type=int, default=-1, help="GN_OPT_XCD_SWIZZLE mask (-1: library default)")
    ap.add_argument("--king-sort", type=int, default=-1, help="GN_OPT_KING_SORT (-1: library default)")
    ap.add_argument("--chain", type=int, default=None, help="GN_OPT_CHAIN (None: library default; -k: exactly k)")
    ap.add_argument("--king-cache", type=int, default=None, help="GN_OPT_KING_CACHE (None: library default)")
    ap.add_argument("--pipeline", type=int, default=None, help="GN_OPT_EXPAND_PIPELINE (None: library default)")
    ap.add_argument("--abi-games", type=int, default=0,
                    help="only the secondary.abi_games line with this many games per GPU (A/B runs)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dropin", action="store_true", help="only the secondary.dropin line (A/B runs)")
    args = ap.parse_args()
    rc = launch_ranks(args.gpus, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.launch_check:
        sys.exit(launch_check())

    c = Ctx(args)
    if args.dropin:
        r = run_dropin(c, 1024, 16, 64, args.check and 32)
        if c.rank == 0:
            print(json.dumps(r), flush=True)
        c.close()
        return
    if args.abi_games:
        r = run_abi_games(c, args.abi_games, 1, args.steps, args.check)
        if c.rank == 0:
            print(json.dumps(r), flush=True)
        c.close()
        return
    G = c.G
    wl = WORKLOADS[args.workload]
    mode = wl["mode"]
    n = args.positions or wl["n"]
    eval_check = max(4096, 16 * args.check) if args.check else 0
    if args.workload == "expand":
        r = run_expand(c, wl, n, args.steps, args.warmup, args.check)
        cfg = {"workload": wl["config"], "games_per_gpu": n, "parents_per_gpu": r["n"],
               "children_per_gpu": r["children"], "evals_per_step_per_gpu": r["n"] + r["children"],
               "evals_per_step_all_gpus": c.world * (r["n"] + r["children"]), "plies": PLIES,
               "ft_rows_per_step_per_gpu": r["rows"], "king_cache_gap_pads": r["scratch_pads"]}
        stage_names = G.EXPAND_STAGES
        data = f"synthetic: seeded random 80-ply games generated on the GPU; nets {c.net_label}"
    else:
        r = run_eval(c, wl, n, args.steps, args.warmup, args.max_plies, eval_check)
        cfg = {"workload": wl["config"], "positions_per_gpu": n, "global_batch": n * c.world,
               "mean_pieces": round(float(r["pieces"].mean()), 3), "max_plies": args.max_plies,
               "ft_rows_per_step_per_gpu": r["rows"]}
        stage_names = EVAL_STAGES
        data = f"synthetic: seeded random-playout positions generated on the GPU; nets {c.net_label}"
    cfg.update({"mode": ["full", "big", "small"][mode], "parallelism": f"dp{c.world} (sharded, no collective)",
                "options": c.options})
    roof = roofline(r["alg"], r["kern_ms"], r["kernel"], load_pmc(args.workload, n, r.get("launches", 1)),
                    r.get("launches", 1))
    roof["stage_ms"] = {k: round(v, 4) for k, v in zip(stage_names, r["stage"])}
    if r.get("plan_ms"):
        roof["plan_kernel_ms"] = round(r["plan_ms"], 4)
    if r.get("finish_ms", 0) > 0.05:
        roof["finish_kernel_ms"] = round(r["finish_ms"], 4)
    elif r.get("plan_ms"):  # (the library's default: the finish runs inside the finalize stage)
        roof["finish"] = "inside finalize (stage_ms.finalize): outputs computed from the slices' partial sums"
    line = {
        "metric": METRIC, "value": round(r["value"], 1), "unit": "evals/s", "n_gpus": c.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["wall"] * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16/int8",
        "data": data, "config": cfg, "roofline": roof,
    }
    # per-rank verification results and checksums (all ranks check their own timed outputs)
    chk = r.get("oracle_check")
    if chk is not None:
        bad = (chk["oracle"]["mismatching_parents"] + (0 if chk["vs_plain_path"]["equal"] else 1)
               if args.workload == "expand" else chk["mismatches"])
        if "gather" in r:
            line["gather"] = r["gather"]
            bad += r["gather"].get("oracle_check", {}).get("mismatching_parents", 0)
        line["oracle_check"] = chk
        line["rank_check_failures"] = c.comm.gather_i64(int(bad))
    line["rank_checksums"] = [f"{x:016x}" for x in c.comm.gather_i64(int(r["checksum"]) & 0x7FFFFFFFFFFFFFFF)]

    if c.rank == 0 and not args.no_cpu_baseline:
        if args.workload == "expand":
            cb = cpu_baseline_expand(c, r["parents"][:1_000_000], mode, args.cpu_seconds)
        else:
            cb = cpu_baseline_eval(c, r["boards"][:200_000], mode, args.cpu_seconds)
        # the whole host beside this GPU's share: not measured (the pool gives one GPU 16 of the
        # host's CPUs), a linear extrapolation to every logical CPU, an upper bound with SMT
        ncpu = os.cpu_count() or cb["cores"]
        cb["whole_host"] = {"value": round(cb["value"] * ncpu / cb["cores"], 1), "unit": cb["unit"], "cores": ncpu,
                            "how": f"linear extrapolation of the {cb['cores']}-thread measurement to all {ncpu} "
                                   f"logical CPUs (not measured; an upper bound with SMT)"}
        line["cpu_baseline"] = cb

    if not args.no_secondary and args.workload == "expand":
        sec = {}
        for name in ("big16m", "small1m"):
            w = WORKLOADS[name]
            # (the small net's launch is < 1 ms: 20 steps after 3 warmups, so that its first launches
            # after the big-net line, with the small table not yet in L2, do not dominate)
            st, wu = (20, 3) if name == "small1m" else (3, 1)
            s = run_eval(c, w, w["n"], st, wu, args.max_plies, 4096 if args.check else 0)
            rf = roofline(s["alg"], s["kern_ms"], s["kernel"], load_pmc(name, w["n"]))
            sec[name] = {"workload": w["config"], "value": round(s["value"], 1), "unit": "evals/s",
                         "kernel": s["kernel"], "kernel_ms": round(s["kern_ms"], 4), "ft_rows": s["rows"],
                         "achieved_GBps": rf["achieved"], "peak_GBps": rf["peak"], "frac": rf["frac"],
                         "traffic": rf["traffic"], "mean_pieces": round(float(s["pieces"].mean()), 3)}
            if "oracle_check" in s:
                sec[name]["oracle_check"] = s["oracle_check"]
                sec[name]["rank_check_failures"] = c.comm.gather_i64(s["oracle_check"]["mismatches"])
        g2 = run_expand2(c, 2048, 1, 2, 256 if args.check else 0)
        if "oracle_check" in g2:
            g2["rank_check_failures"] = c.comm.gather_i64(g2["oracle_check"]["mismatching_children"])
        sec["grandchild"] = g2
        ag = run_abi_games(c, WORKLOADS["expand"]["n"], 1, 2, 256 if args.check else 0)
        ag["frac_of_device_resident"] = round(ag["value"] / line["value"], 4)
        if "oracle_check" in ag:
            ck = ag["oracle_check"]
            ag["rank_check_failures"] = c.comm.gather_i64(ck["oracle"]["mismatching_positions"] +
                                                          ck["vs_device_resident"]["mismatching_games"])
        sec["abi_games"] = ag
        dr = run_dropin(c, 1024, 16, 64, 32 if args.check else 0)
        if "oracle_check" in dr:
            dr["rank_check_failures"] = c.comm.gather_i64(dr["oracle_check"]["mismatches"])
        sec["dropin"] = dr
        line["secondary"] = sec

    if c.rank == 0:
        print(json.dumps(line), flush=True)
    c.close()


if __name__ == "__main__":
    main()
