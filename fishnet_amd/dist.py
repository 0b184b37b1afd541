"""Multi-GPU plumbing for the evaluator: one process per GPU, positions sharded
by rank, RCCL (torch.distributed backend "nccl") used only to broadcast the
.nnue images and to gather per-rank results.  The same code runs
on CPU with the "gloo" backend (tests/test_dist.py)."""
from __future__ import annotations

import os


class ShardComm:
    """collectives: run the torch.distributed collectives (default: only when world > 1; True
    at world 1 drives a one-rank RCCL group through the same calls, tests/test_bench_gpu.py)."""

    def __init__(self, backend: str | None = None, collectives: bool | None = None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.coll = self.world > 1 if collectives is None else collectives
        self.backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        self.device = torch.device("cuda", self.local) if self.backend == "nccl" else torch.device("cpu")
        if self.backend == "nccl":
            torch.cuda.set_device(self.local)
        if self.coll and not dist.is_initialized():
            kw = {"device_id": self.device} if self.backend == "nccl" else {}
            dist.init_process_group(self.backend, **kw)

    # ---- sharding: the library's partitioner (gn_partition), game-aligned ----
    def shard(self, per_rank: int) -> tuple[int, int]:
        """[first, first + per_rank) of the global index space owned by this rank (weak
        scaling: equal weights, so every rank gets per_rank items)."""
        first, last = self.shard_weighted([1] * 0, per_rank * self.world)
        return first, last - first

    def shard_weighted(self, weights, n_items=None) -> tuple[int, int]:
        """[first, last) items of this rank: contiguous ranges cut at item boundaries
        (games), balanced by weight (positions per game); weights empty: equal weights."""
        from fishnet_amd import gpu_nnue
        n = len(weights) if n_items is None else n_items
        b = gpu_nnue.partition(n, self.world, weights if len(weights) else None)
        return b[self.rank], b[self.rank + 1]

    # ---- collectives ---------------------------------------------------------
    def broadcast_bytes(self, data: bytes, src: int = 0) -> bytes:
        if not self.coll:
            return data
        torch, dist = self.torch, self.dist
        ln = torch.tensor([len(data)], dtype=torch.int64, device=self.device)
        dist.broadcast(ln, src)
        if self.rank == src:
            t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.device)
        else:
            t = torch.empty(int(ln.item()), dtype=torch.uint8, device=self.device)
        dist.broadcast(t, src)
        return t.cpu().numpy().tobytes()

    def broadcast_obj(self, obj, src: int = 0):
        if not self.coll:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src)
        return lst[0]

    def barrier(self):
        if self.coll:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.coll:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_i64(self, x: int) -> list[int]:
        if not self.coll:
            return [x]
        t = self.torch.tensor([x & 0x7FFFFFFFFFFFFFFF], dtype=self.torch.int64, device=self.device)
        lst = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(lst, t)
        return [int(v.item()) for v in lst]

    def gather_array(self, arr, dst: int = 0):
        """Gathers numpy arrays of one dtype (e.g. gn_eval records; lengths may differ per
        rank) to dst: the list of every rank's array on dst, None elsewhere."""
        import numpy as np
        if not self.coll:
            return [arr]
        torch, dist = self.torch, self.dist
        data = np.ascontiguousarray(arr).tobytes()
        sizes = self.gather_i64(len(data))
        pad = max(sizes)
        raw = torch.zeros(max(pad, 1), dtype=torch.uint8)
        if data:
            raw[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        raw = raw.to(self.device)
        if self.backend == "nccl":
            lst = [torch.empty_like(raw) for _ in range(self.world)]
            dist.all_gather(lst, raw)
            outs = lst if self.rank == dst else None
        else:
            outs = [torch.empty_like(raw) for _ in range(self.world)] if self.rank == dst else None
            dist.gather(raw, outs, dst=dst)
        if self.rank != dst:
            return None
        return [np.frombuffer(o.cpu().numpy().tobytes()[:sz], dtype=arr.dtype) for o, sz in zip(outs, sizes)]

    def gather_tensor(self, t, dst: int = 0):
        """Gathers a 1-D tensor (device tensors over RCCL, CPU tensors over gloo; the length may
        differ per rank) to dst: dst gets the list of every rank's tensor, the others None.
        This is the result gather of DESIGN.md section 6 (gn_eval records, moves, offsets)."""
        if not self.coll:
            return [t]
        torch, dist = self.torch, self.dist
        sizes = self.gather_i64(int(t.numel()))
        pad = max(sizes)
        if t.numel() < pad:
            buf = torch.zeros(pad, dtype=t.dtype, device=t.device)
            buf[:t.numel()] = t
        else:
            buf = t.contiguous()
        outs = [torch.empty(pad, dtype=t.dtype, device=t.device) for _ in range(self.world)] \
            if self.rank == dst else None
        dist.gather(buf, outs, dst=dst)
        return None if outs is None else [o[:n] for o, n in zip(outs, sizes)]

    def close(self):
        if self.coll and self.dist.is_initialized():
            self.dist.barrier()
            self.dist.destroy_process_group()
