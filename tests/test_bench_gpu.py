"""bench.py's N > 1 code on one GPU: run_expand + gather_results for two
ranks, with a loopback stand-in for ShardComm.  The ranks run one after another in this
process on GPU 0: rank 1 evaluates its shard of games and deposits its records (the gather's
non-root side), rank 0 evaluates its own shard, gathers both, and checks 32 sampled parents of
every rank, with all their children, against the CPU oracle -- exactly the code an 8-GPU run
executes after its timed steps, minus the RCCL transport (two ranks cannot share one GPU
under RCCL).  torch is imported first, as bench.py does, so that its HIP runtime is the one
libgpu_nnue binds to."""
import argparse
import copy
import json
import os

import numpy as np
import torch  # (before libgpu_nnue, as in bench.py)
import pytest

pytestmark = pytest.mark.gpu


class LoopbackHub:
    """What the ranks of one loopback run share: gathered tensors (FIFO per rank, in call order)
    and gathered integers."""

    def __init__(self, world):
        self.world = world
        self.tensors = {r: [] for r in range(world)}
        self.taken = 0
        self.i64 = {r: [] for r in range(world)}


class LoopbackComm:
    """ShardComm's interface for sequential ranks in one process (fishnet_amd/dist.py)."""

    def __init__(self, hub, rank):
        self.hub, self.rank, self.world, self.local = hub, rank, hub.world, 0
        self.backend = "loopback"
        self.device = torch.device("cuda", 0)

    def broadcast_bytes(self, data, src=0):
        return data

    def broadcast_obj(self, obj, src=0):
        return obj

    def barrier(self):
        pass

    def max(self, x):
        return x

    def gather_i64(self, x):
        mine = self.hub.i64[self.rank]
        mine.append(int(x))
        k = len(mine) - 1
        return [self.hub.i64[r][k] if len(self.hub.i64[r]) > k else int(x) for r in range(self.world)]

    def gather_tensor(self, t, dst=0):
        if self.rank != dst:
            self.hub.tensors[self.rank].append(t.clone())
            return None
        k = self.hub.taken
        self.hub.taken += 1
        return [t if r == dst else self.hub.tensors[r][k] for r in range(self.world)]

    def close(self):
        pass


def test_run_expand_and_gather_two_loopback_ranks():
    import bench
    args = argparse.Namespace(swizzle=-1, king_sort=-1, chain=None, king_cache=None)
    hub = LoopbackHub(2)
    c0 = bench.Ctx(args, comm=LoopbackComm(hub, 0))
    c1 = copy.copy(c0)
    c1.comm, c1.rank = LoopbackComm(hub, 1), 1
    wl, games = bench.WORKLOADS["expand"], 48
    try:
        r1 = bench.run_expand(c1, wl, games, 1, 0, 8)
        r0 = bench.run_expand(c0, wl, games, 1, 0, 8)
    finally:
        c0.nn.close()
    for r in (r0, r1):  # each rank's own timed outputs: oracle sample and the plain path
        assert r["oracle_check"]["oracle"]["mismatching_parents"] == 0
        assert r["oracle_check"]["vs_plain_path"]["equal"]
    assert "oracle_check" not in r1["gather"]  # (rank 1 only handed its records to the gather)
    g = r0["gather"]
    assert g["oracle_check"] == {"parents": 64, "ranks": 2, "mismatching_parents": 0,
                                 "of": "the gathered records on rank 0"}
    assert g["bytes_all_ranks"] > 0
    # the two shards are different games
    assert r0["checksum"] != r1["checksum"]


def test_evaluate_device_blocks_until_written(gpu_ctx):
    """gn_evaluate_device is documented as blocking (gpu_nnue.h: the score rule reads
    the in-check count back, so the call synchronises the stream it is given).  On a caller's
    stream the call returns with nothing left queued on that stream and the records written."""
    from fishnet_amd import gpu_nnue as G
    boards = G.random_positions(0x5EED0777, 0, 4096, 160)
    d_b, d_o = gpu_ctx.alloc(boards.nbytes), gpu_ctx.alloc(len(boards) * G.EVAL_SIZE)
    d_b.upload(boards)
    ref = gpu_ctx.evaluate_batch([G.board_to_fen(b) for b in boards], G.MODE_FULL)
    s = torch.cuda.Stream()
    gpu_ctx.evaluate_device(d_b, len(boards), G.MODE_FULL, d_o, stream=s.cuda_stream)
    assert s.query()
    assert np.array_equal(d_o.download(G.EVAL_DTYPE, len(boards)), ref)


_ONE_RANK = r"""
import argparse, json, sys
import torch
sys.path.insert(0, sys.argv[1])
import bench
from fishnet_amd.dist import ShardComm
comm = ShardComm("nccl", collectives=True)  # a one-rank RCCL group, every collective real
c = bench.Ctx(argparse.Namespace(swizzle=-1, king_sort=-1, chain=None, king_cache=None), comm=comm)
r = bench.run_expand(c, bench.WORKLOADS["expand"], 48, 1, 0, 8, gather=True)
print(json.dumps({"oracle": r["oracle_check"]["oracle"]["mismatching_parents"],
                  "plain": r["oracle_check"]["vs_plain_path"]["equal"], "gather": r["gather"]}))
c.nn.close()
comm.close()
"""


def test_rccl_result_gather_one_rank(tmp_path):
    """The result gather's RCCL transport on the GPU (it had never executed): one rank
    in a "nccl" process group with its collectives on (ShardComm(collectives=True)), so the
    nets' broadcast, the length all_gather and the records' torch.distributed.gather all run
    through RCCL on device memory; rank 0 then checks sampled parents of the gathered records,
    with all their children, against the oracle.  In a child process: the process group must
    not outlive the test."""
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    script = tmp_path / "one_rank.py"
    script.write_text(_ONE_RANK)
    p = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["oracle"] == 0 and d["plain"]
    g = d["gather"]
    assert g["oracle_check"]["ranks"] == 1 and g["oracle_check"]["mismatching_parents"] == 0
    assert g["oracle_check"]["parents"] == 32 and g["bytes_all_ranks"] > 0
