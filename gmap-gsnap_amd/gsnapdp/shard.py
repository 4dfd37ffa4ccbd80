"""Multi-GPU plumbing of the benchmark and of batch drivers.

Windows are independent: one read batch is split per read
into contiguous slices balanced by in-band cells (``balanced_ranges``), every
rank aligns its slice against a replicated genome, and the result records +
compact op streams come back to the root rank in ONE collective per batch
(``gather_to_root``: RCCL over xGMI on the GPUs).  One process per GPU;
torch.distributed also carries the start/stop barrier and the max-over-ranks
time.  The same functions run under the ``gloo`` backend on CPU for the tests.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Optional


@dataclass
class Ranks:
    rank: int
    world: int
    local: int
    dist: Optional[object]  # torch.distributed when world > 1


def init_from_env(backend: str = "nccl") -> Ranks:
    """RANK / WORLD_SIZE / LOCAL_RANK from torch.distributed.run; the process
    group is created only for world > 1 (MASTER_ADDR should be 127.0.0.1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return Ranks(rank, world, local, dist)


def shard_seed(base: int, rank: int) -> int:
    """Seed of rank's read shard: disjoint synthetic reads per rank (weak scaling)."""
    return base + rank


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of a fixed batch for rank (strong-scaling drivers)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def balanced_ranges(weights, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) slices of a batch, one per rank, balanced by the
    windows' weights (in-band cells); every window lands in
    exactly one slice and slices follow batch order."""
    import numpy as np
    w = np.asarray(weights, dtype=np.float64)
    n = w.size
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.concatenate([[0.0], np.cumsum(w)])  # cum[c] = weight of windows [0, c)
    cuts = [0]
    for k in range(1, world):
        t = cum[-1] * k / world
        c = int(np.searchsorted(cum, t, side="left"))  # first cut with weight >= t
        if c > 0 and t - cum[c - 1] <= cum[min(c, n)] - t:
            c -= 1
        cuts.append(c)
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(world)]


def gather_to_root(r: Ranks, payload, recv: Optional[list] = None, async_op: bool = False):
    """Gather every rank's payload (equal-size tensors) into `recv` on rank 0:
    one collective (RCCL gather over xGMI on the GPUs, gloo on CPU).  Returns
    the work handle when async_op."""
    if r.dist is None:
        if recv is not None:
            recv[0].copy_(payload)
        return None
    return r.dist.gather(payload, gather_list=recv if r.rank == 0 else None, dst=0, async_op=async_op)


def timed_steps(r: Ranks, step: Callable[[], None], steps: int, sync: Callable[[], None]) -> float:
    """Run exactly `steps` steps bracketed by barrier + sync on both sides and
    return the elapsed seconds, max over ranks."""
    if r.dist is not None:
        r.dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if r.dist is not None:
        r.dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(r, elapsed)


def max_over_ranks(r: Ranks, x: float) -> float:
    if r.dist is None:
        return x
    import torch
    backend = r.dist.get_backend()
    dev = torch.device("cuda", r.local) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    r.dist.all_reduce(t, op=r.dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(units_per_rank_step: int, r: Ranks, steps: int, elapsed: float) -> float:
    """Whole-job throughput: units processed by all ranks / the max time."""
    return r.world * units_per_rank_step * steps / elapsed


def finish(r: Ranks) -> None:
    if r.dist is not None:
        r.dist.barrier()
        r.dist.destroy_process_group()
