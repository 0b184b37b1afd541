"""The N>1 plumbing (fishnet_amd/dist.py) with world_size 2 on CPU ("gloo")."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    try:
        from fishnet_amd import synthnet
        from fishnet_amd.dist import ShardComm
        comm = ShardComm("gloo")
        blob = synthnet.synth_net_bytes(32, 5) if rank == 0 else b""
        got = comm.broadcast_bytes(blob)
        label = comm.broadcast_obj("synthetic" if rank == 0 else None)
        first, count = comm.shard(1000)
        mx = comm.max(float(rank + 1))
        sums = comm.gather_i64(1000 + rank)
        evals = np.zeros(4, dtype=[("psqt", "<i4"), ("positional", "<i4"), ("final_v", "<i4"), ("flags", "<u4")])
        evals["psqt"] = rank
        gathered = comm.gather_array(evals)
        comm.close()
        q.put((rank, len(got), hashlib.sha256(got).hexdigest(), label, first, count, mx, sums,
               None if gathered is None else [int(g["psqt"][0]) for g in gathered]))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, "error", repr(e)))


def test_two_rank_gloo_plumbing():
    import multiprocessing as mp
    from fishnet_amd import synthnet
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        item = q.get(timeout=120)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] != "error" for r in res.values()), res
    blob = synthnet.synth_net_bytes(32, 5)
    for r in (0, 1):
        _, ln, hsh, label, first, count, mx, sums, gathered = res[r]
        assert ln == len(blob) and hsh == hashlib.sha256(blob).hexdigest() and label == "synthetic"
        assert (first, count) == (1000 * r, 1000)
        assert mx == 2.0 and sums == [1000, 1001]
    assert res[0][8] == [0, 1] and res[1][8] is None
