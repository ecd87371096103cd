"""N>1 path on CPU: world_size-2 gloo ranks shard a packet batch with no data-path
collective and aggregate (max time, summed bytes and verify failures) exactly like
bench.py does on RCCL.  The per-rank ICRC work is done by the oracle here (CPU stand-in,
test only); the GPU version of the same loop is bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from icrc_amd.shard import aggregate, shard_range, stream_params


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_stream_params_distinct():
    ps = [stream_params(r) for r in range(8)]
    assert len({p.dqpn for p in ps}) == 8 and len({p.payload_key for p in ps}) == 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "oracle"), os.path.join(root, "open-rdma-driver_amd")]
    import torch.distributed as dist

    import oracle
    from icrc_amd.shard import aggregate, shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 301
    buf, off, lens = oracle.synth_middle_stream(n, pmtu=256)
    lo, hi = shard_range(n, rank, world)
    icrc = oracle.compute_icrc_batch(buf, off[lo:hi], lens[lo:hi])
    # trailers already hold the ICRC; corrupt packets 5, 150, 299 -> 3 verify failures total
    fails = 0
    for i in range(lo, hi):
        p = buf[int(off[i]): int(off[i]) + int(lens[i])].copy()
        if i in (5, 150, 299):
            p[60] ^= 0x10
        fails += 0 if oracle.is_icrc_valid(p) else 1
    gibs, secs, tot_fails = aggregate(int(lens[lo:hi].sum()), 0.5 + rank, fails)
    q.put((rank, lo, hi, icrc.tolist(), gibs, secs, tot_fails))
    dist.destroy_process_group()


def test_gloo_world2_shards_and_aggregates():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle

    buf, off, lens = oracle.synth_middle_stream(301, pmtu=256)
    whole = oracle.compute_icrc_batch(buf, off, lens).tolist()
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 301
    assert res[0][3] + res[1][3] == whole
    for r in res:
        assert r[5] == pytest.approx(1.5)        # max over ranks
        assert r[6] == 3                         # summed failures
        assert r[4] == pytest.approx(int(lens.sum()) / 1.5 / (1 << 30))


def test_aggregate_single_process_identity():
    g, s, f = aggregate(1 << 30, 2.0, 4)
    assert g == pytest.approx(0.5) and s == 2.0 and f == 4
