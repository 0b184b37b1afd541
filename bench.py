#!/usr/bin/env python3
"""bench.py — batched Stockfish NNUE evaluation throughput on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, N>1 under
`torch.distributed.run`; rank 0 prints ONE JSON line.

A "step" is one pass of the hot path over one batch resident in HBM:
  workload big16m (default; BASELINE.json configs[2], the HBM-bound FT gather
  the metric's "% of HBM peak" refers to): GN_MODE_BIG evaluation of
  16,777,216 seeded random-playout positions per GPU, full refresh;
  workload small1m (configs[1]): GN_MODE_SMALL on 1,048,576 positions per GPU;
  workload full16m: the complete Eval::evaluate pipeline (small net, big
  re-evaluation) on 16,777,216 positions per GPU.
Positions are generated on the GPU by the same random-playout code the host
uses (seed 0x5EED0000 + global index), so per-GPU work is fixed as N grows
("scaling": "weak"); there is no data-path collective (positions are
independent).  RCCL (torch.distributed "nccl") is used only to broadcast the
.nnue images from rank 0 and to gather per-rank result checksums + timings.

Nets: GPU_NNUE_BIG / GPU_NNUE_SMALL if set (real Stockfish nets), otherwise the
seeded synthetic nets of identical shape (fishnet_amd/synthnet.py).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "NNUE evals/sec (node) at 1/2/4/8 MI355X + FT gather HBM GB/s as % of peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md (chip table)
SEED = 0x5EED0000
WORKLOADS = {
    "big16m": dict(mode=1, n=1 << 24, l1=3072, config="configs[2]: Stockfish big-net (L1=3072) batch eval of "
                   "16M random-playout positions per MI355X, full refresh (HBM-bound FT gather)"),
    "small1m": dict(mode=2, n=1 << 20, l1=128, config="configs[1]: Stockfish small-net (L1=128) batch eval of "
                    "1M random-playout positions per MI355X"),
    "full16m": dict(mode=0, n=1 << 24, l1=3072, config="Eval::evaluate pipeline (small net, big-net re-eval "
                    "when |nnue| < 236) on 16M random-playout positions per MI355X"),
    "children": dict(mode=1, n=8192, l1=3072, config="configs[3] shape: 8192 random 80-ply games per MI355X "
                     "(81 parents each) x every legal child; GPU movegen + incremental big-net accumulators"),
}
STAGES = ["classify", "small_net", "big_net", "finalize"]


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


def cpu_baseline(G, boards_sample, mode, budget_s):
    """Oracle (CPU restatement, C, -O3 -march=x86-64-v3) on a bounded sample."""
    from fishnet_amd import synthnet
    from oracle import oracle as O
    big_p, small_p, _ = synthnet.net_paths()
    big = O.Net(big_p) if mode != 2 else None
    small = O.Net(small_p) if mode != 1 else None
    threads = max(1, min(16, os.cpu_count() or 1))
    fens = [G.board_to_fen(b) for b in boards_sample]
    done, reps = 0, 0
    t = time.perf_counter()
    while True:  # repeat the sample until the time budget is used (bounded CPU work)
        O.eval_fens(big, small, fens, mode, threads=threads)
        done += len(fens)
        reps += 1
        dt = time.perf_counter() - t
        if dt >= budget_s or reps >= 200:
            break
    return {"value": round(done / dt, 1), "unit": "evals/s", "cores": threads, "kind": "port",
            "sample": f"{len(fens)} positions (first {len(fens)} of rank 0's batch, same nets, same mode) x {reps} "
                      f"passes = {done} evals in {dt:.1f} s; oracle/oracle.c scalar C -O3 -march=x86-64-v3 "
                      f"(AVX2 build class), {threads} POSIX threads on {cpu_model()}"}


def run_children(args, ctx, wl, world, rank, dist, torch, net_label, big_p, small_p, options):
    """configs[3] shape: games x 81 parents, every legal child, incremental."""
    from fishnet_amd import gpu_nnue as G
    games, plies, mode = (args.positions or wl["n"]), 80, wl["mode"]
    n = games * (plies + 1)
    d_par = ctx.alloc(n * 32)
    t = time.perf_counter()
    ctx.random_games_device(SEED, rank * games, games, plies, d_par)
    ctx.synchronize()
    gen_s = time.perf_counter() - t
    if args.warmup:
        ctx.time_expand_device(d_par, n, mode, args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms, children, stages, rows = ctx.time_expand_device(d_par, n, mode, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        w = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    evals = n + children
    value = world * evals * args.steps / wall
    l1 = 3072 if mode != 2 else 128
    stage = 5 if mode != 2 else 4
    alg = rows * (2 * l1 + 4) + n * 32 + children * (24 + 8)
    kern_ms = stages[stage]
    achieved = alg / (kern_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16/int8",
        "data": f"synthetic: seeded random 80-ply games generated on the GPU; nets {net_label}",
        "config": {"workload": wl["config"], "games_per_gpu": games, "parents_per_gpu": n,
                   "children_per_gpu": children, "evals_per_step_per_gpu": evals,
                   "mode": ["full", "big", "small"][mode], "incremental": True,
                   "parallelism": f"dp{world} (games sharded, no collective)", "options": options},
        "roofline": {"bound": "hbm", "kernel": f"expand_eval<{l1}>", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None, "alg_bytes_per_launch": alg, "ft_rows_per_launch": rows,
                     "kernel_ms_per_launch": round(kern_ms, 4),
                     "stage_ms": {k: round(v, 4) for k, v in zip(G.EXPAND_STAGES, stages)}},
        "gen_games_s": round(gen_s, 3),
    }
    if rank == 0 and args.check:
        from oracle import oracle as O
        boards = d_par.download(G.BOARD_DTYPE, n)
        idx = np.linspace(0, n - 1, 24).astype(int)
        fens = [G.board_to_fen(boards[i]) for i in idx]
        parents, offs, moves, kids = ctx.expand_and_evaluate(fens, mode)
        big = O.Net(big_p) if mode != 2 else None
        small = O.Net(small_p) if mode != 1 else None
        bad = 0
        for i, fen in enumerate(fens):
            _, m_exp, k_exp = O.expand_eval(big, small, fen, mode)
            got = dict(zip(moves[offs[i]:offs[i + 1]].tolist(), map(tuple, kids[offs[i]:offs[i + 1]].tolist())))
            bad += got != dict(zip(m_exp, map(tuple, k_exp.tolist())))
        line["oracle_check"] = {"parents": len(fens), "children": int(offs[-1]), "mismatching_parents": bad}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    d_par.free()
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="big16m")
    ap.add_argument("--positions", type=int, default=0, help="override positions per GPU")
    ap.add_argument("--max-plies", type=int, default=160)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--check", type=int, default=2048, help="positions re-checked against the oracle (rank 0)")
    ap.add_argument("--swizzle", type=int, default=1, help="GN_OPT_XCD_SWIZZLE")
    ap.add_argument("--king-sort", type=int, default=-1, help="GN_OPT_KING_SORT (-1: library default)")
    args = ap.parse_args()

    import torch  # first: torch's HIP runtime is the one libgpu_nnue then binds to
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from fishnet_amd import build, gpu_nnue as G, synthnet
    build.build()
    wl = WORKLOADS[args.workload]
    n = args.positions or wl["n"]
    mode = wl["mode"]

    # ---- nets: rank 0 reads, RCCL broadcast over xGMI, every rank loads from memory
    big_p, small_p, net_label = synthnet.net_paths() if rank == 0 else (None, None, None)
    blobs = []
    for path in (big_p, small_p):
        data = open(path, "rb").read() if rank == 0 else b""
        if world > 1:
            ln = torch.tensor([len(data)], dtype=torch.int64, device="cuda")
            dist.broadcast(ln, 0)
            t = (torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda() if rank == 0
                 else torch.empty(int(ln.item()), dtype=torch.uint8, device="cuda"))
            dist.broadcast(t, 0)
            data = t.cpu().numpy().tobytes()
        blobs.append(data)
    if world > 1:
        lab = [net_label]
        dist.broadcast_object_list(lab, 0)
        net_label = lab[0]
    ctx = G.GpuNnue(big_bytes=blobs[0], small_bytes=blobs[1], devices=[local])
    ctx.set_option(G.OPT_XCD_SWIZZLE, args.swizzle)
    if args.king_sort >= 0:
        ctx.set_option(G.OPT_KING_SORT, args.king_sort)
    options = {"xcd_swizzle": ctx.get_option(G.OPT_XCD_SWIZZLE), "king_sort": ctx.get_option(G.OPT_KING_SORT)}

    def run_workload(mode, n, steps, warmup, measure_roofline):
        d_boards = ctx.alloc(n * 32)
        d_out = ctx.alloc(n * 16)
        t = time.perf_counter()
        ctx.random_positions_device(SEED, rank * n, n, args.max_plies, d_boards)
        ctx.synchronize()
        gen_s = time.perf_counter() - t
        for _ in range(warmup):
            ctx.evaluate_device(d_boards, n, mode, d_out)
        ctx.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ms_events, per_kernel = ctx.time_evaluate_device(d_boards, n, mode, d_out, steps, per_kernel=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        if world > 1:
            w = torch.tensor([wall], dtype=torch.float64, device="cuda")
            dist.all_reduce(w, op=dist.ReduceOp.MAX)
            wall = float(w.item())
        out = d_out.download(G.EVAL_DTYPE, n)
        boards = d_boards.download(G.BOARD_DTYPE, n)
        res = dict(wall=wall, ms_events=ms_events, per_kernel=per_kernel, gen_s=gen_s, out=out, boards=boards)
        d_boards.free()
        d_out.free()
        return res

    if args.workload == "children":
        run_children(args, ctx, wl, world, rank, dist, torch, net_label, big_p, small_p, options)
        return

    r = run_workload(mode, n, args.steps, args.warmup, True)
    total = world * n * args.steps
    value = total / r["wall"]
    pieces = popcounts(r["boards"]["occ"])
    row_bytes = 2 * wl["l1"] + 4  # one feature: L1 int16 weights + the bucket's int32 PSQT weight
    stage = {0: 2, 1: 2, 2: 1}[mode]  # dominant kernel: big net, or the small net in small-only mode
    if mode == 0:
        need_big = int(np.count_nonzero((r["out"]["flags"] & 2) == 0))
        gathered = int(pieces[(r["out"]["flags"] & 2) == 0].sum())
        alg_bytes = 2 * gathered * row_bytes + need_big * 40
    else:
        alg_bytes = 2 * int(pieces.sum()) * row_bytes + n * 40
    kern_ms = r["per_kernel"][stage]
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "r01", "pmc_summary_big16m.json")
    if args.workload == "big16m" and n == WORKLOADS["big16m"]["n"] and os.path.exists(pmc):
        traffic = json.load(open(pmc))["hbm_side_bytes_per_launch"]
        traffic_src = ("profiles/r01/pmc_summary_big16m.json: rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE "
                       "of eval_net<3072>, separate --pmc passes of this workload; L2-miss bytes (MALL + HBM)")
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    # result gather: per-rank checksum of the outputs (RCCL gather of a tiny tensor)
    csum = int(np.bitwise_xor.reduce(r["out"].view(np.uint32).astype(np.uint64) * np.uint64(2654435761)))
    checks = [csum]
    if world > 1:
        t = torch.tensor([csum & 0x7FFFFFFFFFFFFFFF], dtype=torch.int64, device="cuda")
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        checks = [int(x.item()) for x in lst]

    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(r["wall"] * 1e3 / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int16/int8",
        "data": f"synthetic: seeded random-playout positions generated on the GPU; nets {net_label}",
        "config": {"workload": wl["config"], "positions_per_gpu": n, "global_batch": n * world,
                   "mode": ["full", "big", "small"][mode], "mean_pieces": round(float(pieces.mean()), 3),
                   "max_plies": args.max_plies, "parallelism": f"dp{world} (positions sharded, no collective)",
                   "options": options},
        "roofline": {"bound": "hbm", "kernel": f"eval_net<{wl['l1']}> ({STAGES[stage]})",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": alg_bytes, "kernel_ms_per_launch": round(kern_ms, 4),
                     "stage_ms": {k: round(v, 4) for k, v in zip(STAGES, r["per_kernel"])}},
        "gen_positions_s": round(r["gen_s"], 3),
        "rank_checksums": checks,
    }

    # bit-exactness spot check of this very batch against the oracle (rank 0)
    if rank == 0 and args.check:
        from oracle import oracle as O
        k = min(args.check, n)
        fens = [G.board_to_fen(b) for b in r["boards"][:k]]
        big = O.Net(big_p) if mode != 2 else None
        small = O.Net(small_p) if mode != 1 else None
        exp = O.eval_fens(big, small, fens, mode, threads=max(1, min(16, os.cpu_count() or 1)))
        line["oracle_check"] = {"positions": k, "mismatches": int(np.count_nonzero(exp != r["out"][:k]))}

    if rank == 0 and not args.no_cpu_baseline:
        k = min(n, 200_000)
        line["cpu_baseline"] = cpu_baseline(G, r["boards"][:k], mode, args.cpu_seconds)

    if not args.no_secondary and args.workload == "big16m":
        s = run_workload(2, 1 << 20, max(args.steps, 5), args.warmup, False)
        sp = popcounts(s["boards"]["occ"])
        sb = 2 * int(sp.sum()) * (2 * 128 + 4) + (1 << 20) * 40
        line["secondary"] = {"workload": WORKLOADS["small1m"]["config"],
                             "value": round(world * (1 << 20) * max(args.steps, 5) / s["wall"], 1),
                             "unit": "evals/s",
                             "small_net_kernel_ms": round(s["per_kernel"][1], 4),
                             "small_net_alg_GBps": round(sb / (s["per_kernel"][1] * 1e-3) / 1e9, 1)}

    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
