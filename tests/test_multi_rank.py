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
    gibs, secs, tot_fails, tot_bytes = aggregate(int(lens[lo:hi].sum()), 0.5 + rank, fails)
    q.put((rank, lo, hi, icrc.tolist(), gibs, secs, tot_fails, tot_bytes))
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
        assert r[7] == int(lens.sum())                # summed bytes


def test_aggregate_single_process_identity():
    g, s, f, b = aggregate(1 << 30, 2.0, 4)
    assert g == pytest.approx(0.5) and s == 2.0 and f == 4 and b == 1 << 30


# ---- bench.py's own launcher and aggregation (world 2, gloo, CPU stand-in step) ----------------
import json  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB_L = 28 + 28 + 256 + 4  # --pmtu 256


def _bench(*extra, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-stub", "--pmtu", "256",
                        "--steps", "2", "--warmup", "1", *extra],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_launcher_world2_weak():
    rc, res, err = _bench("--gpus", "2", "--packets", "48")
    assert rc == 0, err[-2000:]
    assert res["n_gpus"] == 2 and res["scaling"] == "weak"
    assert res["config"]["bytes_total_per_step"] == 2 * 48 * STUB_L  # summed over both ranks
    assert res["config"]["packets_per_gpu"] == 48
    assert res["parity_sample"]["failures_all_ranks"] == 0
    pr = res["per_rank"]  # every rank's own time and device, gathered outside the timed region
    assert pr["device"] == [0, 1] and len(pr["kernel_ms"]) == 2 and len(pr["wall_ms_per_step"]) == 2
    assert pr["kernel_ms_min"] == min(pr["kernel_ms"]) and pr["kernel_ms_max"] == max(pr["kernel_ms"])


def test_bench_launcher_world2_strong():
    rc, res, err = _bench("--gpus", "2", "--packets", "65", "--scaling", "strong")
    assert rc == 0, err[-2000:]
    assert res["n_gpus"] == 2 and res["scaling"] == "strong"
    assert res["config"]["bytes_total_per_step"] == 65 * STUB_L  # a fixed total, split 33 + 32
    assert res["config"]["packets_per_gpu"] == 33  # rank 0's shard (shard_range)


def test_bench_launcher_sums_failures_and_fails():
    rc, res, err = _bench("--gpus", "2", "--packets", "16", "--inject-fault-rank", "1")
    assert rc != 0
    assert res["parity_sample"]["failures_all_ranks"] == 1


def test_bench_launcher_kills_stalled_ranks():
    """A rank that never reaches the first barrier: the launcher's --launch-timeout kills the whole
    rank group (torchrun + ranks, one session) and exits 3 with a one-line JSON error, well inside
    the driver's own limit."""
    import time

    t0 = time.monotonic()
    rc, res, err = _bench("--gpus", "2", "--packets", "8", "--stall-rank", "1", "--dist-timeout", "600",
                          "--launch-timeout", "20")
    assert rc == 3, err[-2000:]
    assert res["value"] is None and "timed out" in res["error"]
    assert time.monotonic() - t0 < 120


def test_bench_collective_timeout_ends_ranks():
    """The same stall with a short --dist-timeout: the waiting rank's barrier raises (gloo honours the
    process-group timeout), torchrun tears the group down, and bench exits non-zero."""
    import time

    t0 = time.monotonic()
    rc, res, err = _bench("--gpus", "2", "--packets", "8", "--stall-rank", "1", "--dist-timeout", "8",
                          "--launch-timeout", "200")
    assert rc not in (0, 3), err[-2000:]
    assert time.monotonic() - t0 < 150


def test_bench_refuses_world_size_mismatch():
    rc, res, _ = _bench("--gpus", "2", "--packets", "8", env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert rc == 2 and res is None


def test_bench_single_rank_stub():
    rc, res, err = _bench("--packets", "8")
    assert rc == 0, err[-2000:]
    assert res["n_gpus"] == 1 and res["config"]["bytes_total_per_step"] == 8 * STUB_L


def test_gpu_count_without_hip(tmp_path, monkeypatch):
    """bench.py's launcher counts GPUs from the KFD topology (GPU nodes: simd_count > 0) and amdsmi
    (the smaller count), capped by the visibility variables; it never calls HIP, and with no
    source at all it refuses loudly."""
    from icrc_amd import shard

    monkeypatch.setattr(shard, "amdsmi_gpu_count", lambda: None)

    nodes = tmp_path / "nodes"
    for i, simd in enumerate([0, 304, 304, 0, 304]):  # two CPU nodes, three GPU agents
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ngfx_target_version 90500\n")
    assert shard.visible_gpu_count({}, str(nodes)) == (3, "kfd-topology")
    assert shard.visible_gpu_count({"HIP_VISIBLE_DEVICES": "1"}, str(nodes))[0] == 1
    assert shard.visible_gpu_count({"ROCR_VISIBLE_DEVICES": "0,1", "HIP_VISIBLE_DEVICES": "0"}, str(nodes))[0] == 1
    assert shard.visible_gpu_count({"CUDA_VISIBLE_DEVICES": "0,1,2,3,4,5"}, str(nodes))[0] == 3
    with pytest.raises(RuntimeError):
        shard.visible_gpu_count({}, str(tmp_path / "absent"))
    monkeypatch.setattr(shard, "amdsmi_gpu_count", lambda: 1)  # amdsmi sees fewer: it wins
    assert shard.visible_gpu_count({}, str(nodes)) == (1, "amdsmi")


def test_bench_launcher_refuses_without_gpu_count():
    """Without --cpu-stub, --gpus 2 on a machine where neither the KFD topology nor amdsmi shows
    two GPUs exits 2 before starting any rank."""
    from icrc_amd import shard

    try:
        have, _ = shard.visible_gpu_count()
    except RuntimeError:
        have = 0
    if have >= 2:
        pytest.skip("this machine has 2 GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120, cwd=ROOT)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "torch.distributed.run" not in p.stderr


def test_time_steps_settles_before_warmup(monkeypatch):
    """bench.time_steps: untimed repetitions for --settle-ms before the W warm-up steps (GPU runs
    only: the cpu stub skips it), then exactly K timed steps."""
    sys.path.insert(0, ROOT)
    import bench

    calls = {"n": 0}

    def step():
        calls["n"] += 1

    bench.ARGS = bench.parse(["--settle-ms", "30", "--steps", "5", "--warmup", "2"])
    assert bench.ARGS.settle_ms == 30.0 and not bench.ARGS.dist_rehearsal
    monkeypatch.setattr(bench.ARGS, "cpu_stub", True)  # no torch.cuda events on the CPU
    bench.time_steps(step, 5, 2, 1, lambda: None, None)
    assert calls["n"] == 7  # the stub skips the settle phase
    monkeypatch.setattr(bench.ARGS, "cpu_stub", False)
    calls["n"] = 0

    class _Ev:  # stand-in for torch.cuda.Event (no GPU here)
        def __init__(self, **kw):
            pass

        def record(self):
            pass

        def elapsed_time(self, other):
            return 1.0

    import torch

    monkeypatch.setattr(torch.cuda, "Event", _Ev)
    t0 = __import__("time").perf_counter()
    wall, kms = bench.time_steps(step, 5, 2, 1, lambda: None, None)
    assert __import__("time").perf_counter() - t0 >= 0.03
    assert calls["n"] > 7 and (calls["n"] - 7) % 4 == 0  # settle bursts of 4, then 2 + 5
    assert kms == 1.0 / 5
