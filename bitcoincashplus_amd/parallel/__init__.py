"""One-process-per-GPU scale-out over ``torch.distributed``.

On MI355X nodes the backend is ``"nccl"`` (RCCL over xGMI); CPU tests use ``gloo``.
The reference has no multi-device path (its solver loop is a single CPU thread,
reference src/rpc/mining.cpp:161-199, and script checks fan out over threads,
src/checkqueue.h); here the two embarrassingly parallel hot paths scale across GPUs:

* **Nonce-space data parallel mining** (``DistributedEquihashMiner``): every rank
  solves a disjoint nonce lane (rank id in the top nonce word), solution counts are
  summed with one all-reduce per step, and ``mine`` stops all ranks as soon as any
  rank finds a solution meeting the target (all-reduce MIN over the winning rank,
  then a broadcast of its solution from that rank).
* **Sharded batch verification** (``sharded_verify``): a batch of checks (ECDSA
  triples, Equihash solutions) is split into contiguous shards, each rank verifies
  its shard on its own GPU, and the per-item verdicts are all-gathered as one uint8
  tensor — one collective per batch, sized for the point-to-point xGMI ring.
"""
from __future__ import annotations

import os
import struct
from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist


def world() -> tuple:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def init_from_env(backend: Optional[str] = None) -> tuple:
    """Initialise the process group from torchrun's env (MASTER_ADDR should be
    127.0.0.1 on a single node). Picks nccl (RCCL) when a GPU is visible."""
    rank, size = world()
    if size > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return world()


def _device() -> torch.device:
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard_bounds(n: int, rank: int, size: int) -> tuple:
    """Contiguous [lo, hi) shard of n items for `rank` (first n % size ranks get one more)."""
    base, extra = divmod(n, size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def nonce_bytes(counter: int, rank: int, lane: int = 0) -> bytes:
    """32-byte Equihash nonce: counter in word 0, lane in word 1, rank in word 3 —
    disjoint across ranks by construction."""
    return struct.pack("<QQQQ", counter, lane, 0, rank)


def sharded_verify(items: Sequence, verify_shard: Callable[[Sequence], Sequence[bool]]) -> List[bool]:
    """Verify `items` across all ranks; every rank returns the full verdict list.
    `verify_shard` runs on this rank's contiguous shard (e.g. ops.ecdsa_verify)."""
    rank, size = world()
    if size == 1 or not dist.is_initialized():
        return [bool(x) for x in verify_shard(items)]
    lo, hi = shard_bounds(len(items), rank, size)
    local = [bool(x) for x in verify_shard(items[lo:hi])] if hi > lo else []
    width = -(-len(items) // size)
    dev = _device()
    buf = torch.zeros(width, dtype=torch.uint8, device=dev)
    if local:
        buf[: len(local)] = torch.tensor(local, dtype=torch.uint8, device=dev)
    out = [torch.empty_like(buf) for _ in range(size)]
    dist.all_gather(out, buf)
    res: List[bool] = []
    for r in range(size):
        rlo, rhi = shard_bounds(len(items), r, size)
        res.extend(bool(v) for v in out[r][: rhi - rlo].tolist())
    return res


class DistributedEquihashMiner:
    """Nonce-space data-parallel Equihash miner.

    backend="gpu" uses the gfx950 batch solver (EquihashModel.gpu_solver);
    backend="cpu" uses the native CPU solver (tests / hosts without a GPU).
    `header` is the CEquihashInput prefix (header without nonce and solution).
    """

    def __init__(self, n: int, k: int, header: bytes, batch: int = 8, backend: str = "gpu", device: int = 0):
        from ..models import EquihashModel

        self.model = EquihashModel(n, k)
        self.header = bytes(header)
        self.batch = batch
        self.backend = backend
        self.rank, self.size = world()
        self.solver = self.model.gpu_solver(batch, device) if backend == "gpu" else None
        self.counter = 0

    def _states(self, base: int):
        sts = []
        for b in range(self.batch):
            nonce = nonce_bytes(base + b, self.rank)
            sts.append((nonce, self.model.state(self.header + nonce)))
        return sts

    def step(self):
        """Solve one batch of this rank's nonces. Returns [(nonce, [solutions])]."""
        sts = self._states(self.counter)
        self.counter += self.batch
        if self.solver is not None:
            sols = self.solver.solve([s for _, s in sts])
        else:
            sols = [self.model.solve_cpu(s) for _, s in sts]
        return [(nonce, list(ss)) for (nonce, _), ss in zip(sts, sols)]

    def step_count(self) -> int:
        """One step on every rank; returns the job-wide solution count."""
        local = sum(len(s) for _, s in self.step())
        t = torch.tensor([local], dtype=torch.int64, device=_device())
        if self.size > 1 and dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    def mine(self, accept: Callable[[bytes, bytes], bool], max_steps: int = 1000):
        """Run steps until some rank finds (nonce, solution) with accept(...) true.
        All ranks return the same winner (lowest winning rank), or None."""
        dev = _device()
        sol_len = self.model.solution_bytes
        for _ in range(max_steps):
            found = None
            for nonce, sols in self.step():
                for s in sols:
                    if accept(nonce, s):
                        found = (nonce, s)
                        break
                if found:
                    break
            if self.size == 1 or not dist.is_initialized():
                if found:
                    return found
                continue
            flag = torch.tensor([self.rank if found else self.size], dtype=torch.int64, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            winner = int(flag.item())
            if winner == self.size:
                continue
            payload = torch.zeros(32 + sol_len, dtype=torch.uint8, device=dev)
            if winner == self.rank:
                payload.copy_(torch.frombuffer(bytearray(found[0] + found[1]), dtype=torch.uint8).to(dev))
            dist.broadcast(payload, src=winner)
            raw = bytes(payload.cpu().tolist())
            return raw[:32], raw[32:]
        return None


__all__ = ["init_from_env", "world", "shard_bounds", "nonce_bytes", "sharded_verify", "DistributedEquihashMiner"]
