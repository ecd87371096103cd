"""Multi-GPU sharding for the ICRC path: packets are independent, so the work
splits with no data-path collective.  One process per GPU; the only cross-rank steps are
the timing barrier, a max over per-rank times and a host-side sum of counters.

    weak scaling   (configs[4]): rank r owns its own QP stream (dqpn = 2 + r)
    strong scaling             : a fixed batch split into contiguous packet ranges

The reference's own concurrency model is the same shape: independent per-thread callers with
no shared state (blue-rdma-device/src/device_inner.rs:119-171).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import NamedTuple


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) packet range of `rank`; sizes differ by at most one packet."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


@dataclass(frozen=True)
class StreamParams:
    dqpn: int
    payload_key: int
    psn0: int


def stream_params(rank: int) -> StreamParams:
    """Per-rank independent QP stream (weak scaling)."""
    return StreamParams(dqpn=2 + rank, payload_key=0x5EED5EED + rank, psn0=0)


class Aggregate(NamedTuple):
    gib_per_s: float    # whole-job: bytes of every rank / the slowest rank's time
    seconds: float      # max over ranks
    failures: int       # sum over ranks
    total_bytes: int    # sum over ranks


def aggregate(bytes_local: int, seconds_local: float, failures_local: int, group=None) -> Aggregate:
    """Whole-job (GiB/s, max seconds, total failures, total bytes) across ranks; identity when
    not distributed.  Uses torch.distributed (nccl on GPUs, gloo on CPU): one MAX and one SUM
    all-reduce of a few scalars, outside any timed region."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return Aggregate(bytes_local / seconds_local / float(1 << 30), seconds_local, failures_local, bytes_local)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([seconds_local], dtype=torch.float64, device=dev)
    c = torch.tensor([bytes_local, failures_local], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(c, op=dist.ReduceOp.SUM, group=group)
    secs = float(t.item())
    total_bytes, fails = (int(x) for x in c.tolist())
    return Aggregate(total_bytes / secs / float(1 << 30), secs, fails, total_bytes)
