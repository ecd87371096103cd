"""Multi-GPU sharding for the ICRC path: packets are independent, so the work
splits with no data-path collective.  One process per GPU; the only cross-rank steps are
the timing barrier, a max over per-rank times and a host-side sum of counters.

    weak scaling   (configs[4]): rank r owns its own QP stream (dqpn = 2 + r)
    strong scaling             : a fixed batch split into contiguous packet ranges

The reference's own concurrency model is the same shape: independent per-thread callers with
no shared state (blue-rdma-device/src/device_inner.rs:119-171).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import NamedTuple, Optional


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


def gather_floats(values, group=None) -> list:
    """Every rank's list of floats (same length on every rank), rank-ordered; [values] when not
    distributed.  One all-gather of a small tensor, outside any timed region (per-rank kernel
    times and device ordinals for the rank-0 line)."""
    import torch
    import torch.distributed as dist

    vals = [float(v) for v in values]
    if not (dist.is_available() and dist.is_initialized()):
        return [vals]
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [o.cpu().tolist() for o in out]


# ---- GPU count for the launcher, without initialising HIP in the launching process ----------
_VISIBILITY_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _visible_limit(env) -> Optional[int]:
    """How many devices the visibility variables leave (None = unrestricted).  HIP applies
    ROCR_VISIBLE_DEVICES first, then HIP_ / CUDA_VISIBLE_DEVICES on what remains: each set
    variable caps the count at its number of entries."""
    limit = None
    for var in _VISIBILITY_VARS:
        v = env.get(var)
        if v is None:
            continue
        n = len([x for x in v.split(",") if x.strip() != ""])
        limit = n if limit is None else min(limit, n)
    return limit


def kfd_gpu_count(sysfs: str = "/sys/class/kfd/kfd/topology/nodes") -> Optional[int]:
    """GPU agents in the KFD topology (nodes whose `simd_count` is nonzero; CPU nodes have 0).
    None when the topology cannot be read."""
    try:
        nodes = os.listdir(sysfs)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(sysfs, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    return n


def amdsmi_gpu_count() -> Optional[int]:
    """GPUs amdsmi enumerates (through the kernel driver, not HIP).  None if amdsmi is absent or
    fails to initialise."""
    try:
        import amdsmi
    except Exception:
        return None
    try:
        amdsmi.amdsmi_init()
    except Exception:
        return None
    try:
        return len(amdsmi.amdsmi_get_processor_handles())
    except Exception:
        return None
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:
            pass


def visible_gpu_count(env=None, sysfs: str = "/sys/class/kfd/kfd/topology/nodes") -> tuple[int, str]:
    """(GPUs this process may use, how it was counted) — the KFD topology and amdsmi (the smaller
    count when both answer), capped by the visibility variables.  Never calls HIP: bench.py's launcher uses it before starting the
    ranks, so the parent process does not initialise a GPU.  Raises RuntimeError when neither
    source works (no silent fallback to a HIP call)."""
    env = os.environ if env is None else env
    found = [(c, name) for c, name in ((kfd_gpu_count(sysfs), "kfd-topology"), (amdsmi_gpu_count(), "amdsmi"))
             if c is not None]
    if not found:
        raise RuntimeError("cannot count GPUs without HIP: no KFD topology at %s and amdsmi unavailable" % sysfs)
    # both sources when both answer: the smaller count (a container may see the host's topology
    # nodes while only some GPUs are its own)
    n, how = min(found)
    lim = _visible_limit(env)
    if lim is not None and lim < n:
        n, how = lim, how + "+visible-devices"
    return n, how
