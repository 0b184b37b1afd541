#!/usr/bin/env python3
"""bench.py — batched Stockfish NNUE evaluation throughput on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, N>1 under
`torch.distributed.run`; rank 0 prints ONE JSON line.

Default workload `expand` (BASELINE.json configs[4], the 1/2/4/8-GPU scaling
configuration; configs[3]'s batch shape): every GPU holds 49,152 random 80-ply
games = 3,981,312 parent positions (81 per game), and one step is
  legal-child generation (GPU bitboard movegen, count + scan + write with
  per-child FT deltas) + big-net evaluation of every parent and every legal
  child (parents refreshed once, children incremental from the parent
  accumulators) + the Eval::evaluate epilogue,
~127 M evaluated positions per GPU per step, i.e. >= 1e9 per step on 8 GPUs.
Secondary results (same JSON object, not `value`):
  big16m  configs[2]: big-net full refresh of 16,777,216 positions per GPU;
  small1m configs[1]: small-net evaluation of 1,048,576 positions per GPU.

All inputs are generated on the GPU by the same seeded playout code the host
uses (`value` never includes host transfers), per-GPU work is fixed as N grows
("scaling": "weak"), and there is no data-path collective: RCCL
(torch.distributed "nccl") only broadcasts the .nnue images from rank 0 and
gathers per-rank checksums / the max wall time.  Nets: GPU_NNUE_BIG /
GPU_NNUE_SMALL if set (real Stockfish nets), else seeded synthetic nets of
identical shape (fishnet_amd/synthnet.py).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NNUE evals/sec (node) at 1/2/4/8 MI355X + FT gather HBM GB/s as % of peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md, chip table)
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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


class Ctx:
    """Per-rank state: library context + the RCCL plumbing of fishnet_amd/dist.py."""

    def __init__(self, args):
        import torch  # first: torch's HIP runtime is then the one libgpu_nnue binds to
        from fishnet_amd.dist import ShardComm
        self.torch = torch
        self.comm = ShardComm("nccl")
        self.rank, self.world, self.local = self.comm.rank, self.comm.world, self.comm.local
        from fishnet_amd import build, gpu_nnue as G, synthnet
        build.build()
        self.G = G
        # nets: rank 0 reads, RCCL broadcast over xGMI, every rank loads from memory
        big_p, small_p, label = synthnet.net_paths() if self.rank == 0 else (None, None, None)
        blobs = [self.comm.broadcast_bytes(open(p, "rb").read() if self.rank == 0 else b"") for p in (big_p, small_p)]
        self.big_p, self.small_p = big_p, small_p
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
        self.options = {"xcd_swizzle": self.nn.get_option(G.OPT_XCD_SWIZZLE),
                        "king_sort": self.nn.get_option(G.OPT_KING_SORT),
                        "incremental_children": self.nn.get_option(G.OPT_INCREMENTAL_CHILDREN),
                        "chain": self._opt(G.OPT_CHAIN), "king_cache": self._opt(G.OPT_KING_CACHE)}

    def _opt(self, option):
        try:
            return self.nn.get_option(option)
        except self.G.GnError:  # an older library (A/B runs through GPU_NNUE_LIB)
            return None

    def barrier_sync(self):
        self.comm.barrier()
        self.torch.cuda.synchronize()

    def max_over_ranks(self, x: float) -> float:
        return self.comm.max(x)

    def gather_checksums(self, c: int):
        return self.comm.gather_i64(c)

    def close(self):
        self.comm.close()
        self.nn.close()


def checksum(arr: np.ndarray) -> int:
    return int(np.bitwise_xor.reduce(arr.view(np.uint32).astype(np.uint64) * np.uint64(2654435761)))


def run_eval(c: Ctx, wl: dict, n: int, steps: int, warmup: int, max_plies: int):
    """Full-refresh batch evaluation of n device-resident positions per GPU."""
    G, nn, mode = c.G, c.nn, wl["mode"]
    d_b, d_o = nn.alloc(n * 32), nn.alloc(n * 16)
    t = time.perf_counter()
    first, _ = c.comm.shard(n)
    nn.random_positions_device(SEED, first, n, max_plies, d_b)
    nn.synchronize()
    gen_s = time.perf_counter() - t
    for _ in range(warmup):
        nn.evaluate_device(d_b, n, mode, d_o)
    nn.synchronize()
    c.barrier_sync()
    t0 = time.perf_counter()
    _, stage = nn.time_evaluate_device(d_b, n, mode, d_o, steps, per_kernel=True)
    c.barrier_sync()
    wall = c.max_over_ranks(time.perf_counter() - t0)
    out, boards = d_o.download(G.EVAL_DTYPE, n), d_b.download(G.BOARD_DTYPE, n)
    d_b.free(), d_o.free()
    pieces = popcounts(boards["occ"])
    row = 2 * wl["l1"] + 4  # one feature: L1 int16 weights + the bucket's int32 PSQT weight
    if mode == 0:
        big = (out["flags"] & G.FLAG_SMALLNET) == 0
        alg = 2 * int(pieces[big].sum()) * row + int(big.sum()) * 40
    else:
        alg = 2 * int(pieces.sum()) * row + n * 40
    k = 1 if mode == 2 else 2
    return dict(value=c.world * n * steps / wall, wall=wall, stage=stage, kern_ms=stage[k], alg=alg, out=out,
                boards=boards, pieces=pieces, gen_s=gen_s,
                kernel=f"eval_net<{wl['l1']}> ({EVAL_STAGES[k]})")


def run_expand(c: Ctx, wl: dict, games: int, steps: int, warmup: int):
    """Games x 81 parents, every legal child, incremental evaluation."""
    G, nn, mode = c.G, c.nn, wl["mode"]
    n = games * (PLIES + 1)
    d_p = nn.alloc(n * 32)
    t = time.perf_counter()
    first, _ = c.comm.shard(games)
    nn.random_games_device(SEED, first, games, PLIES, d_p)
    nn.synchronize()
    gen_s = time.perf_counter() - t
    if warmup:
        nn.time_expand_device(d_p, n, mode, warmup)
    c.barrier_sync()
    t0 = time.perf_counter()
    _, children, stage, rows = nn.time_expand_device(d_p, n, mode, steps)
    c.barrier_sync()
    wall = c.max_over_ranks(time.perf_counter() - t0)
    parents = d_p.download(G.BOARD_DTYPE, n)
    d_p.free()
    l1 = wl["l1"]
    alg = rows * (2 * l1 + 4) + n * 32 + children * (24 + 8)
    k = 5 if mode != 2 else 4
    return dict(value=c.world * (n + children) * steps / wall, wall=wall, stage=stage, kern_ms=stage[k], alg=alg,
                rows=rows, parents=parents, n=n, children=children, gen_s=gen_s, kernel=f"expand_stream<{l1}>" if l1 != 128 else f"expand_eval<{l1}>")


def oracle_threads():
    return max(1, min(16, os.cpu_count() or 1))


def cpu_baseline_eval(c: Ctx, boards, mode, budget_s):
    """Oracle (CPU restatement, scalar C -O3 -march=x86-64-v3) on a bounded sample."""
    from oracle import oracle as O
    big = O.Net(c.big_p) if mode != 2 else None
    small = O.Net(c.small_p) if mode != 1 else None
    th = oracle_threads()
    fens = [c.G.board_to_fen(b) for b in boards]
    done, reps, t = 0, 0, time.perf_counter()
    while True:
        O.eval_fens(big, small, fens, mode, threads=th)
        done, reps = done + len(fens), reps + 1
        dt = time.perf_counter() - t
        if dt >= budget_s or reps >= 200:
            break
    return {"value": round(done / dt, 1), "unit": "evals/s", "cores": th, "kind": "port",
            "sample": f"{len(fens)} positions of rank 0's batch x {reps} passes = {done} evals in {dt:.1f} s; "
                      f"oracle/oracle.c scalar C -O3 -march=x86-64-v3 (AVX2 build class), {th} threads, {cpu_model()}"}


def cpu_baseline_expand(c: Ctx, parents, mode, budget_s):
    """Oracle: every parent + every legal child (make-move + full refresh) on a bounded sample."""
    from oracle import oracle as O
    big = O.Net(c.big_p) if mode != 2 else None
    small = O.Net(c.small_p) if mode != 1 else None
    th = oracle_threads()
    done, t = 0, time.perf_counter()
    with cf.ThreadPoolExecutor(th) as ex:  # ctypes releases the GIL inside the C call
        for k in range(0, len(parents), th * 8):  # FEN text per chunk (the oracle's input), timed with it
            fens = [c.G.board_to_fen(b) for b in parents[k:k + th * 8]]
            done += sum(1 + len(r[1]) for r in ex.map(lambda f: O.expand_eval(big, small, f, mode), fens))
            if time.perf_counter() - t >= budget_s:
                break
    dt = time.perf_counter() - t
    return {"value": round(done / dt, 1), "unit": "evals/s", "cores": th, "kind": "port",
            "sample": f"{done} evals (parents of rank 0's games + all their legal children) in {dt:.1f} s; "
                      f"oracle/oracle.c (mailbox movegen, full-refresh NNUE) scalar C -O3 -march=x86-64-v3, "
                      f"{th} threads, {cpu_model()}"}


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
    ap.add_argument("--check", type=int, default=1024, help="positions / parents re-checked against the oracle")
    ap.add_argument("--swizzle", type=int, default=-1, help="GN_OPT_XCD_SWIZZLE mask (-1: library default)")
    ap.add_argument("--king-sort", type=int, default=-1, help="GN_OPT_KING_SORT (-1: library default)")
    ap.add_argument("--chain", type=int, default=None, help="GN_OPT_CHAIN (None: library default; -k: exactly k)")
    ap.add_argument("--king-cache", type=int, default=None, help="GN_OPT_KING_CACHE (None: library default)")
    args = ap.parse_args()

    c = Ctx(args)
    G = c.G
    wl = WORKLOADS[args.workload]
    mode = wl["mode"]
    n = args.positions or wl["n"]
    if args.workload == "expand":
        r = run_expand(c, wl, n, args.steps, args.warmup)
        cfg = {"workload": wl["config"], "games_per_gpu": n, "parents_per_gpu": r["n"],
               "children_per_gpu": r["children"], "evals_per_step_per_gpu": r["n"] + r["children"],
               "evals_per_step_all_gpus": c.world * (r["n"] + r["children"]), "plies": PLIES,
               "ft_rows_per_step_per_gpu": r["rows"]}
        stage_names = G.EXPAND_STAGES
        data = f"synthetic: seeded random 80-ply games generated on the GPU; nets {c.net_label}"
    else:
        r = run_eval(c, wl, n, args.steps, args.warmup, args.max_plies)
        cfg = {"workload": wl["config"], "positions_per_gpu": n, "global_batch": n * c.world,
               "mean_pieces": round(float(r["pieces"].mean()), 3), "max_plies": args.max_plies}
        stage_names = EVAL_STAGES
        data = f"synthetic: seeded random-playout positions generated on the GPU; nets {c.net_label}"
    cfg.update({"mode": ["full", "big", "small"][mode], "parallelism": f"dp{c.world} (sharded, no collective)",
                "options": c.options})
    achieved = r["alg"] / (r["kern_ms"] * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": round(r["value"], 1), "unit": "evals/s", "n_gpus": c.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["wall"] * 1e3 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16/int8",
        "data": data, "config": cfg,
        "roofline": {"bound": "hbm", "kernel": r["kernel"], "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "alg_bytes_per_launch": r["alg"], "kernel_ms_per_launch": round(r["kern_ms"], 4),
                     "stage_ms": {k: round(v, 4) for k, v in zip(stage_names, r["stage"])}},
    }
    pmc = os.path.join(ROOT, "profiles", "latest_pmc.json")
    if os.path.exists(pmc):
        p = json.load(open(pmc)).get(args.workload)
        if p and p.get("positions") == n:
            line["roofline"]["traffic"] = p["hbm_side_bytes_per_launch"]
            line["roofline"]["traffic_source"] = p["source"]

    if c.rank == 0 and args.check:
        from oracle import oracle as O
        big = O.Net(c.big_p) if mode != 2 else None
        small = O.Net(c.small_p) if mode != 1 else None
        if args.workload == "expand":
            idx = np.linspace(0, r["n"] - 1, min(args.check, 64)).astype(int)
            fens = [G.board_to_fen(r["parents"][i]) for i in idx]
            _, offs, moves, kids = c.nn.expand_and_evaluate(fens, mode)
            bad = 0
            for i, fen in enumerate(fens):
                _, m_exp, k_exp = O.expand_eval(big, small, fen, mode)
                got = dict(zip(moves[offs[i]:offs[i + 1]].tolist(), map(tuple, kids[offs[i]:offs[i + 1]].tolist())))
                bad += got != dict(zip(m_exp, map(tuple, k_exp.tolist())))
            line["oracle_check"] = {"parents": len(fens), "children": int(offs[-1]), "mismatching_parents": bad}
        else:
            k = min(args.check, n)
            fens = [G.board_to_fen(b) for b in r["boards"][:k]]
            exp = O.eval_fens(big, small, fens, mode, threads=oracle_threads())
            line["oracle_check"] = {"positions": k, "mismatches": int(np.count_nonzero(exp != r["out"][:k]))}
    if "out" in r:
        line["rank_checksums"] = c.gather_checksums(checksum(r["out"]))

    if c.rank == 0 and not args.no_cpu_baseline:
        if args.workload == "expand":
            line["cpu_baseline"] = cpu_baseline_expand(c, r["parents"][:400_000], mode, args.cpu_seconds)
        else:
            line["cpu_baseline"] = cpu_baseline_eval(c, r["boards"][:200_000], mode, args.cpu_seconds)

    if not args.no_secondary and args.workload == "expand":
        sec = {}
        for name in ("big16m", "small1m"):
            w = WORKLOADS[name]
            s = run_eval(c, w, w["n"], 3, 1, args.max_plies)
            a = s["alg"] / (s["kern_ms"] * 1e-3) / 1e9
            sec[name] = {"workload": w["config"], "value": round(s["value"], 1), "unit": "evals/s",
                         "kernel": s["kernel"], "kernel_ms": round(s["kern_ms"], 4), "achieved_GBps": round(a, 1),
                         "frac_of_hbm_peak": round(a / HBM_PEAK_GBS, 4),
                         "mean_pieces": round(float(s["pieces"].mean()), 3)}
        line["secondary"] = sec

    if c.rank == 0:
        print(json.dumps(line), flush=True)
    c.close()


if __name__ == "__main__":
    main()
