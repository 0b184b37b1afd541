"""The N>1 path (fishnet_amd/dist.py) with world_size 2 on CPU ("gloo"): the net
broadcast, the library's partitioner (gn_partition) cutting game-aligned shards,
every rank evaluating its own shard (the CPU oracle stands in for the rank's GPU),
and rank 0 checking the gathered results against a single-process evaluation."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# three short lichess-shaped batches (root FEN + UCI moves) of different lengths
GAMES = [
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", "e2e4 c7c5 g1f3 d7d6 d2d4 c5d4 f3d4 g8f6 b1c3 a7a6"),
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", "d2d4 d7d5 c2c4 e7e6"),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", "e1g1 e8c8 a2a3 b4c3 d2c3"),
    ("4k3/8/8/8/8/8/4P3/4K3 w - - 0 1", "e2e4 e8d7 e4e5 d7e6 e1e2"),
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _game_fens(O):
    return [O.replay_game(root, moves)[0] for root, moves in GAMES]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    try:
        from fishnet_amd import synthnet
        from fishnet_amd.dist import ShardComm
        from oracle import oracle as O
        comm = ShardComm("gloo")
        blob = open(synthnet.cached_synth_net(128, 2), "rb").read() if rank == 0 else b""
        got = comm.broadcast_bytes(blob)
        label = comm.broadcast_obj("synthetic" if rank == 0 else None)
        first, count = comm.shard(1000)
        mx = comm.max(float(rank + 1))
        sums = comm.gather_i64(1000 + rank)
        # this rank's games (weights = positions per game), evaluated with the net it received
        games = _game_fens(O)
        g0, g1 = comm.shard_weighted([len(g) for g in games])
        net = O.Net(data=got)
        mine = [f for g in games[g0:g1] for f in g]
        evals = O.eval_fens(None, net, mine, O.MODE_SMALL) if mine else np.zeros(0, dtype=O.EVAL_DTYPE)
        gathered = comm.gather_array(evals)
        # the bench's result gather (gather_tensor: device tensors over RCCL there, CPU tensors
        # over gloo here): the records as raw bytes, lengths differing per rank
        import torch
        tens = comm.gather_tensor(torch.from_numpy(np.ascontiguousarray(evals).view(np.uint8).copy()))
        comm.close()
        q.put((rank, len(got), hashlib.sha256(got).hexdigest(), label, first, count, mx, sums, (g0, g1),
               None if gathered is None else np.concatenate(gathered).tobytes(),
               None if tens is None else b"".join(t.numpy().tobytes() for t in tens)))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, "error", repr(e)))


def test_two_rank_gloo_shards_evaluate():
    import multiprocessing as mp
    from fishnet_amd import synthnet
    from oracle import oracle as O
    O.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=180)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res.values()), res
    blob = open(synthnet.cached_synth_net(128, 2), "rb").read()
    for r in (0, 1):
        _, ln, hsh, label, first, count, mx, sums, _, _, _ = res[r]
        assert ln == len(blob) and hsh == hashlib.sha256(blob).hexdigest() and label == "synthetic"
        assert (first, count) == (1000 * r, 1000)
        assert mx == 2.0 and sums == [1000, 1001]
    # game-aligned shards covering every game once, balanced by positions (11+5 | 6+6)
    assert res[0][8] == (0, 2) and res[1][8] == (2, 4)
    games = _game_fens(O)
    exp = O.eval_fens(None, O.Net(data=blob), [f for g in games for f in g], O.MODE_SMALL)
    assert res[0][9] == exp.tobytes() and res[1][9] is None
    assert res[0][10] == exp.tobytes() and res[1][10] is None


def test_partition_is_game_aligned_and_balanced():
    from fishnet_amd import gpu_nnue as G
    assert G.partition(10, 3) == [0, 4, 7, 10]
    assert G.partition(8, 8) == list(range(9)) and G.partition(0, 4) == [0, 0, 0, 0, 0]
    w = [81] * 5 + [3] * 50 + [200]
    b = G.partition(len(w), 4, w)
    assert b[0] == 0 and b[-1] == len(w) and all(x <= y for x, y in zip(b, b[1:]))
    tot = sum(w)
    for k in range(1, 4):  # shard k starts at the first game whose prefix reaches k/4 of the positions
        assert sum(w[:b[k]]) >= -(-tot * k // 4) and (b[k] == 0 or sum(w[:b[k] - 1]) < -(-tot * k // 4))


def _bench(args, env):
    import subprocess
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=240)


def test_bench_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` without a launcher (WORLD_SIZE unset) starts two ranks itself
    (torch.distributed.run as a child process, before any GPU work), each with WORLD_SIZE=2;
    --launch-check makes the ranks meet over gloo instead of doing GPU work."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = _bench(["--gpus", "2", "--launch-check"], env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line == {"world": 2, "ranks": [[0, 0], [1, 1]]}


def test_bench_world_size_mismatch_fails():
    """Under a launcher, WORLD_SIZE must equal --gpus: a mismatch exits 2 before any GPU work."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = _bench(["--gpus", "1", "--launch-check"], env)
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in p.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = _bench(["--gpus", "1", "--launch-check"], env)  # one rank, no launcher: runs in place
    assert p.returncode == 0 and '"world": 1' in p.stdout


def _gather_worker(rank, world, port, q):
    """One rank of the world-size-4 record gather: this rank's expansion outputs as CPU tensors of
    the sizes the library writes (gn_eval records, u32 offsets, u16 moves), a different number of
    parents and children per rank, through bench.gather_records (ShardComm.gather_tensor over
    gloo; RCCL on device tensors in an 8-GPU run)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    try:
        import types
        import torch
        import bench
        from fishnet_amd import gpu_nnue as G
        from fishnet_amd.dist import ShardComm
        comm = ShardComm("gloo")
        n, children = _gather_shape(rank)
        out = {k: types.SimpleNamespace(tensor=torch.from_numpy(v.copy())) for k, v in _gather_bytes(rank).items()}
        c = types.SimpleNamespace(G=G, torch=torch, comm=comm)
        got, nbytes = bench.gather_records(c, out, n, children)
        comm.close()
        q.put((rank, nbytes, None if got["po"] is None else
               {k: [t.numpy().tobytes() for t in v] for k, v in got.items()}))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, "error", repr(e)))


def _gather_shape(rank):
    return 81 * (rank + 1) + 7 * rank, 2_000 + 977 * rank  # (parents, children) of this rank


def _gather_bytes(rank):
    """Deterministic record bytes of one rank (the library's record sizes, ABI v4)."""
    from fishnet_amd import gpu_nnue as G
    n, ch = _gather_shape(rank)
    rng = np.random.default_rng(900 + rank)
    return {"po": rng.integers(0, 256, n * G.EVAL_SIZE, dtype=np.uint8),
            "off": np.sort(rng.integers(0, ch + 1, n + 1)).astype(np.uint32).view(np.uint8),
            "mv": rng.integers(0, 256, ch * 2, dtype=np.uint8),
            "co": rng.integers(0, 256, ch * G.EVAL_SIZE, dtype=np.uint8)}


def test_four_rank_gloo_record_gather():
    """bench.py's result gather (gather_records, the code an N-GPU run executes
    after its timed steps) at world size 4 with a different record count per rank: rank 0 gets
    every rank's parent records, offsets, child moves and child records byte for byte, the
    other ranks None, and every rank the total byte count."""
    import multiprocessing as mp
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res.values()), res
    exp = [_gather_bytes(r) for r in range(world)]
    total = sum(len(v) for e in exp for v in e.values())
    for r in range(world):
        assert res[r][1] == total
        assert (res[r][2] is None) == (r != 0)
    for k in ("po", "off", "mv", "co"):
        assert res[0][2][k] == [exp[r][k].tobytes() for r in range(world)], k
