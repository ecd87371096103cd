#!/usr/bin/env python3
"""bench.py — device-resident ICRC throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1 Mi x 4 KiB-MTU RDMA WRITE_MIDDLE packets (L = 4156 B:
IPv4 20 + UDP 8 + BTH 12 + RETH 16 + 4096 payload + ICRC 4), synthesised on the device with
the reference's PacketWriter field layout; one "step" = one ICRC-compute pass (kernel launch)
over the whole batch, inputs resident in HBM, ICRCs written to an HBM array.

Multi-GPU (configs[4]): one process per GPU, no collective on the data path.
  * `python bench.py --gpus N` with no WORLD_SIZE in the environment starts
    `python -m torch.distributed.run --nproc-per-node N ... bench.py ...` as a CHILD process
    (before anything touches a GPU) and exits with its status; under torch.distributed.run
    WORLD_SIZE must equal --gpus, and every rank must have a GPU of its own, or bench exits
    non-zero.
  * --scaling weak (default): every rank runs its own independent QP stream of --packets
    packets (dqpn = 2 + rank).  --scaling strong: --packets packets in total, split into
    contiguous shards (shard.shard_range) of one stream.
  * value = bytes of every rank / the slowest rank's time (shard.aggregate: one MAX and one
    SUM all-reduce of scalars, outside the timed region).

Every rank checks a sample of its ICRCs against the CPU restatement (oracle/, the checker;
outside the timed region); the failures are summed over ranks and bench exits 1 if any.

Prints ONE JSON line (rank 0).  value = whole-job GiB/s of packet bytes (sum of L, which
equals the algorithmic bytes: L-4 read + 4 written per packet).  roofline = the ICRC kernel's
achieved GB/s (HIP events on the launch stream) vs the 8.0 TB/s HBM3E peak.  cpu_baseline =
the CPU port of compute_icrc with a crc32fast-equivalent PCLMULQDQ core (oracle/icrc_fast.c),
rank 0 / N=1 only, on a bounded sample of the same packets.

Every GPU measurement repeats its step untimed for --settle-ms (150) before its W warm-up steps:
the first ~30 launches in a fresh process run slower while the clocks settle (rocprof trace of
the plain bench: 0.67 -> 0.76 -> 0.677 ms over launches 1-25).

--cpu-stub (tests only): the same launcher, rank handling, barriers and aggregation on gloo
with a CPU stand-in step (zlib.crc32 of every packet, not the ICRC and not the product), so
the N>1 plumbing is exercised on a machine without GPUs (tests/test_multi_rank.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)
METRIC = "device-resident ICRC GiB/s over 4 KiB-MTU packet batches; % of HBM-read roofline"


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="before the W warm-up steps of every GPU measurement, repeat the step for this "
                         "long (untimed): a fresh process's first ~30 launches of the C1 kernel run up "
                         "to 12 %% slower while the GPU's clocks settle (profiles/r04_clock_settle/)")
    ap.add_argument("--packets", type=int, default=1 << 20,
                    help="packets per GPU (weak scaling) or in total (strong scaling)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--pmtu", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline time budget")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (the parity sample still runs)")
    ap.add_argument("--check-packets", type=int, default=2048,
                    help="per rank: packets at each end of the shard checked against the CPU restatement")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the configs[2] / configs[3] legs of the default line (N = 1)")
    ap.add_argument("--only", choices=("c2", "rx", "msg", "host"), default=None,
                    help="run one secondary leg alone and print it: c2 = the configs[2] kernel (rocprofv3 --pmc "
                         "passes), rx = the short-packet / configs[2] receive legs, msg = the per-message host legs, "
                         "host = the host-resident (PCIe) rate")
    ap.add_argument("--extra", action="store_true",
                    help="also time verify, trailer stores, mixed-MTU, 16 MiB round trip, packetizer, receive "
                         "parse and the host-resident path")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds: process-group init and every collective / barrier (N > 1)")
    ap.add_argument("--launch-timeout", type=float, default=540.0,
                    help="seconds: the launcher kills the whole rank group and exits 3 when the ranks have not "
                         "finished by then (N > 1)")
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="initialise the RCCL process group (barriers, all-reduce, all-gather) even at world "
                         "size 1: rehearses the N > 1 path on a one-GPU box (run under torch.distributed.run)")
    ap.add_argument("--cpu-stub", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--inject-fault-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stall-rank", type=int, default=-1, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---- launcher ------------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_module():
    """icrc_amd/shard.py loaded on its own: importing the icrc_amd package would load the HIP
    library (its static constructors register kernels) in the launching process."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "_icrc_shard_launcher", os.path.join(ROOT, "open-rdma-driver_amd", "icrc_amd", "shard.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod  # dataclasses resolve their module through sys.modules
    spec.loader.exec_module(mod)
    return mod


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 without torch.distributed.run around us: start it as a child process (no
    exec, nothing has touched a GPU here: the GPUs are counted from the KFD topology or amdsmi,
    never through HIP) and return its exit status."""
    if not args.cpu_stub:
        try:
            have, how = _shard_module().visible_gpu_count()
        except RuntimeError as e:
            log(f"bench.py: {e}; refusing to launch {args.gpus} ranks")
            return 2
        if have < args.gpus:
            log(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible ({how}); refusing to report a "
                f"{have}-GPU number as {args.gpus}")
            return 2
        log(f"bench.py: {have} GPU(s) visible ({how})")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    # a collective that outlives --dist-timeout raises on its rank instead of blocking forever
    env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    log("bench.py: launching " + " ".join(cmd[1:]))
    # its own session: on expiry the whole group (torchrun + every rank) is killed, never re-exec'd
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return p.wait(timeout=args.launch_timeout)
    except subprocess.TimeoutExpired:
        import signal

        for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        log(f"bench.py: the {args.gpus} ranks did not finish within --launch-timeout {args.launch_timeout:g} s; "
            "killed their process group")
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": args.gpus,
                          "error": f"ranks timed out after {args.launch_timeout:g} s (killed)"}), flush=True)
        return 3


def _dist_timeout(args):
    from datetime import timedelta

    return timedelta(seconds=args.dist_timeout)


# ---- timing --------------------------------------------------------------------------------
def time_steps(fn, steps: int, warmup: int, world: int, sync, barrier):
    """Warmup, barrier + sync, K timed steps, sync + barrier.  Returns (this rank's wall seconds,
    kernel ms per step from HIP events on the launch stream or None)."""
    if ARGS is not None and not ARGS.cpu_stub and ARGS.settle_ms > 0:
        # untimed: launches in bursts of 4 until settle_ms of wall time, so the timed steps see the
        # steady clocks and not the power-management transient of the first launches
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < ARGS.settle_ms:
            for _ in range(4):
                fn()
            sync()
    for _ in range(warmup):
        fn()
    sync()
    if barrier is not None:
        barrier()
    sync()
    ev = None
    if not ARGS.cpu_stub:
        import torch

        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    if ev:
        ev[0].record()
    for _ in range(steps):
        fn()
    if ev:
        ev[1].record()
    sync()
    if barrier is not None:
        barrier()
    sync()
    wall = time.perf_counter() - t0
    return wall, (ev[0].elapsed_time(ev[1]) / steps if ev else None)


def time_kernel(fn, steps: int, warmup: int, world: int):
    """GPU launches: (wall seconds of this rank, kernel ms per launch)."""
    import torch
    import torch.distributed as dist

    return time_steps(fn, steps, warmup, world, torch.cuda.synchronize, dist.barrier if dist.is_initialized() else None)


ARGS = None


def main(argv=None) -> int:
    global ARGS
    argv = sys.argv[1:] if argv is None else argv
    args = ARGS = parse(argv)
    if args.gpus < 1:
        log("bench.py: --gpus must be >= 1")
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
        return 2
    if os.environ.get("BENCH_DUMP_MAPS"):  # diagnostics: the address map at the end of the Python exit path
        import atexit
        import shutil

        atexit.register(shutil.copyfile, "/proc/self/maps", os.environ["BENCH_DUMP_MAPS"])
    if args.cpu_stub:
        return run_cpu_stub(args, rank, world)
    return run_gpu(args, rank, world, local)


# ---- the GPU run ---------------------------------------------------------------------------
def run_gpu(args, rank: int, world: int, local: int) -> int:
    import torch
    import torch.distributed as dist

    if local >= torch.cuda.device_count():
        log(f"bench.py: rank {rank} (local {local}) has no GPU of its own "
            f"({torch.cuda.device_count()} visible)")
        return 2
    torch.cuda.set_device(local)
    if args.dist_rehearsal and "MASTER_ADDR" not in os.environ:  # not under torch.distributed.run
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    if world > 1 or args.dist_rehearsal:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=_dist_timeout(args))
    import icrc_amd
    from icrc_amd import shard, workloads

    eng = icrc_amd.Engine(local)
    if eng.ordinal != local:
        log(f"bench.py: rank {rank}: engine on device {eng.ordinal}, expected LOCAL_RANK {local}")
        return 2
    stream = torch.cuda.current_stream().cuda_stream
    if args.only == "c2":
        import oracle as orc

        leg, fails = config_c2(eng, stream, args, world, orc)
        print(json.dumps({"configs": {"c2": leg}}), flush=True)
        return 1 if fails else 0
    if args.only == "rx":
        rx = receive_short(eng, stream, args, world)
        print(json.dumps(rx), flush=True)
        return 0 if all(v["all_ok"] and not v.get("parity_failures") for v in rx.values()) else 1
    if args.only == "msg":
        msg = host_message_c0(eng, stream, args)
        print(json.dumps(msg), flush=True)
        return 0
    if args.only == "host":
        hr = host_resident(eng, stream, args)
        print(json.dumps(hr), flush=True)
        return 0 if hr.get("host_resident_results_match_device", False) else 1

    # ---- C1 workload: weak = one QP stream per rank; strong = a shard of one stream ----
    if args.scaling == "weak":
        sp = shard.stream_params(rank)
        w = workloads.write_middle_stream(args.packets, args.pmtu, dqpn=sp.dqpn, payload_key=sp.payload_key)
    else:
        lo, hi = shard.shard_range(args.packets, rank, world)
        w = workloads.subset(workloads.write_middle_stream(args.packets, args.pmtu), lo, hi)
    n = w.n
    L = int(w.lens[0])
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def step():
        eng.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), False, stream)

    wall, kms = time_kernel(step, args.steps, args.warmup, world)
    bytes_per_step = n * L
    # SURVEY 8(d) secondary denominator, same box and batch, after the timed region: the
    # kernel's loads-only build (variant 19 of the A/B library: the same row loads, ring and waits,
    # no CRC), into a scratch array (its results are wrong by design)
    ab = icrc_amd.Engine(local, lib=icrc_amd.ab_library())
    ab.set_variant(LOADS_ONLY_VARIANT)
    d_scratch = torch.zeros(n, dtype=torch.int32, device="cuda")
    _, loads_ms = time_kernel(lambda: ab.compute_strided(d_buf.data_ptr(), L, L, n, d_scratch.data_ptr(), False, stream),
                              min(args.steps, 20), 3, world)
    torch.cuda.synchronize()
    ab.close()
    del d_scratch
    per_rank = shard.gather_floats([kms, eng.ordinal, wall / args.steps * 1e3, loads_ms])

    # ---- CPU leg (outside the timed region): the parity sample on every rank; the CPU
    # baseline on rank 0 at N = 1.  The oracle is the checker / CPU port here only. ----
    import oracle as orc

    fails, checked = check_sample(orc, d_buf, d_out, n, L, args.check_packets, rank, args.inject_fault_rank)
    agg = shard.aggregate(bytes_per_step * args.steps, wall, fails)
    achieved = bytes_per_step / (kms * 1e-3) / 1e9

    result = {
        "metric": METRIC,
        "value": round(agg.gib_per_s, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(agg.seconds / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-synthesised RDMA WRITE_MIDDLE packets, splitmix64 payload)",
        "config": {
            "workload": ("configs[1]: 1Mi x 4KiB-MTU packets per GPU, device-resident ICRC compute"
                         if world == 1 else
                         f"configs[4]: {world} independent QP streams, one per GPU, {args.packets} packets each"
                         if args.scaling == "weak" else
                         f"configs[4] strong scaling: {args.packets} packets of one stream split {world} ways"),
            "packets_per_gpu": n,
            "packets_total_per_step": agg.total_bytes // args.steps // L,
            "packet_bytes": L,
            "pmtu": args.pmtu,
            "bytes_per_gpu_per_step": bytes_per_step,
            "bytes_total_per_step": agg.total_bytes // args.steps,
            "parallelism": f"shard-per-gpu x{world} (no collective on the data path)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "icrc_batch_kernel<kCompute> (rank 0)",
            "kernel_ms": round(kms, 4),
            "achievable": {
                "GB/s": round(bytes_per_step / (loads_ms * 1e-3) / 1e9, 1),
                "kernel_ms": round(loads_ms, 4),
                "frac": round(loads_ms / kms, 4),
                "source": "the same kernel's loads-only build (variant 19 of the A/B library "
                          "libicrc_amd_ab.so: same row loads and ring, no CRC) on the same batch, timed after "
                          "the K steps; frac = achieved / achievable",
            },
        },
        "parity_sample": {"packets_checked_per_rank": checked, "failures_all_ranks": agg.failures},
        "per_rank": per_rank_fields(per_rank),
    }
    tr = pmc_traffic(n, L)
    if tr is not None:
        result["roofline"]["traffic"] = tr["traffic_bytes"]
        result["roofline"]["traffic_source"] = (
            f"profiles/{PMC_TRAFFIC_FILE}: {tr['kernel']} HBM bytes per launch (FETCH_SIZE x "
            f"{tr['fetch_correction']} + WRITE_SIZE), {tr['ratio_to_algorithmic']}x the algorithmic bytes")

    if rank == 0 and world == 1 and not args.no_cpu:
        host = d_buf[: min(n, 16384) * L].cpu().numpy()
        result["cpu_baseline"], result["cpu_context"] = cpu_baseline(orc, host, L, d_out, args)

    cfg_fails = 0
    if world == 1 and not args.no_configs:  # configs[2] and [3] after the headline (value untouched)
        del d_buf, d_out
        torch.cuda.empty_cache()
        c2, f2 = config_c2(eng, stream, args, world, orc)
        c3, f3 = config_c3(eng, stream, args, world, orc)
        c2rx, f2rx = config_c2_rx(eng, stream, args, world, orc)
        result["configs"] = {"c2": c2, "c3": c3, "c2_rx": c2rx}
        cfg_fails += f2rx
        c0 = config_c0_native()
        if c0 is not None:
            result["configs"]["c0_msg"] = c0
            cfg_fails += 0 if c0.get("bad", 1) == 0 else 1
        cfg_fails += f2 + f3

    if args.extra:
        result["extra"] = extra_measurements(eng, stream, args, world)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if agg.failures or cfg_fails:
        log(f"bench.py: {agg.failures + cfg_fails} ICRC mismatches against the CPU restatement")
        return 1
    return 0


def config_c2(eng, stream, args, world, orc):
    """configs[2] in the default line: the mixed-MTU batch (4 Mi packets, 256 B / 1 KiB / 4 KiB
    payload classes, P ~ k^-1.5, 10 % ragged LAST packets; 1.82 GB) through the default ragged
    dispatch (one hybrid launch), timed like the headline (settle, warm-up, HIP events on the launch
    stream).  Its traffic ratio comes from the committed PMC record of this build's oct / long-packet
    sources (PMC_C2_FILE), or is null.  Parity: 4096 packets (both ends of the batch) against the
    CPU restatement.  Returns (leg, mismatches)."""
    import torch

    from icrc_amd import workloads

    wm = workloads.mixed_mtu_stream(4 << 20)
    d_buf = workloads.synthesize(eng, wm, stream=stream)
    d_off, d_len = dev(wm.off), dev(wm.lens)
    d_out = torch.zeros(wm.n, dtype=torch.int32, device="cuda")
    _, kms = time_kernel(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n,
                                                   d_out.data_ptr(), False, 0, stream),
                         min(args.steps, 20), min(args.warmup, 5), world)
    tot = int(wm.lens.astype(np.uint64).sum())
    got = d_out.cpu().numpy().view(np.uint32)
    fails = 0
    for a, b in ((0, 2048), (wm.n - 2048, wm.n)):
        lo, hi = int(wm.off[a]), int(wm.off[b - 1]) + int(wm.lens[b - 1])
        host = d_buf[lo:hi].cpu().numpy()
        want = orc.compute_icrc_batch(host, (wm.off[a:b] - np.uint64(lo)).astype(np.uint64), wm.lens[a:b])
        fails += int(np.count_nonzero(got[a:b] != want))
    leg = {"workload": "configs[2]: 4 Mi mixed-MTU packets (256 B / 1 KiB / 4 KiB classes, power-law, 10 % ragged), "
                       "ragged (offset, length) arrays, one hybrid launch",
           "packets": wm.n, "bytes": tot, "kernel_ms": round(kms, 4),
           "GiB/s": round(tot / (kms * 1e-3) / GIB, 1),
           "frac": round(tot / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic_ratio": None, "parity_checked": 4096, "parity_failures": fails}
    tr = pmc_record(PMC_C2_FILE, C2_SOURCES, wm.n, None)
    if tr is not None:
        leg["traffic_ratio"] = tr["ratio_to_algorithmic"]
        leg["traffic_source"] = f"profiles/{PMC_C2_FILE} ({tr['kernel']}: FETCH_SIZE x {tr['fetch_correction']} + WRITE_SIZE)"
    del d_buf, d_off, d_len, d_out
    torch.cuda.empty_cache()
    return leg, fails


def config_c3(eng, stream, args, world, orc):
    """configs[3] in the default line: one 16 MiB RDMA WRITE segmented at PMTU 4096 (4096 packets,
    Write::handle's FIRST / MIDDLE... / LAST), compute with write_trailer (send) then verify with
    zero_trailer (receive) per round trip; every trailer checked against the CPU restatement once.
    Returns (leg, mismatches)."""
    import torch

    from icrc_amd import workloads

    w3 = workloads.write_message(16 << 20, 4096)
    d_buf = workloads.synthesize(eng, w3, stream=stream)
    host0 = d_buf.cpu().numpy()
    want = orc.compute_icrc_batch(host0, w3.off, w3.lens)
    d_off, d_len = dev(w3.off), dev(w3.lens)
    d_out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    d_ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def rt():
        eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_out.data_ptr(), True, 0, stream)
        eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_ok.data_ptr(), True, 0, stream)

    _, kms = time_kernel(rt, min(args.steps, 20), min(args.warmup, 5), world)
    # Each direction's GPU time per launch: 16 launches of one kind queued behind a spin kernel
    # (torch.cuda._sleep), so the host has enqueued all of them before the GPU reaches the first and
    # the events see the GPU's own rate (dispatch and the gaps between kernels included, the host's
    # ~9 us per launch from Python not).
    def gpu_rate(fn, k=16, reps=5):
        out = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(4_000_000)
            e0.record()
            for _ in range(k):
                fn()
            e1.record()
            e1.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3 / k)
        return float(np.median(out))

    k_us = {"compute": gpu_rate(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n,
                                                         d_out.data_ptr(), True, 0, stream)),
            "verify": gpu_rate(lambda: eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n,
                                                        d_ok.data_ptr(), True, 0, stream))}
    eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_out.data_ptr(), True, 0, stream)
    eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_ok.data_ptr(), True, 0, stream)
    torch.cuda.synchronize()
    fails = int(np.count_nonzero(d_out.cpu().numpy().view(np.uint32) != want))
    all_ok = bool((d_ok == 1).all().item())
    tot3 = int(w3.lens.astype(np.uint64).sum())
    leg = {"workload": "configs[3]: 16 MiB RDMA WRITE at PMTU 4096 (4096 packets), compute + write_trailer then "
                       "verify + zero_trailer",
           "packets": w3.n, "ms_per_roundtrip": round(kms, 4),
           "GiB/s_per_direction": round(2 * tot3 / (kms * 1e-3) / GIB, 1),
           "frac": round(2 * tot3 / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "frac_note": "per direction: packet bytes / (round trip / 2) / 8 TB/s (HIP events over back-to-back "
                        "launches: the two kernels and the gaps between them)",
           "gpu_us_per_launch": {"compute_write_trailer": round(k_us["compute"], 2),
                                 "verify_zero_trailer": round(k_us["verify"], 2)},
           "gpu_frac": {k: round(tot3 / (v * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) for k, v in
                        (("compute_write_trailer", k_us["compute"]), ("verify_zero_trailer", k_us["verify"]))},
           "gpu_note": "16 launches of one direction queued behind a spin kernel, events around them: the GPU's "
                       "own rate per launch (dispatch and inter-kernel gaps in it, host launch cost not); DESIGN "
                       "§6 decomposes it (an empty kernel of this grid: ~2.5 us)",
           "all_ok": all_ok, "parity_checked": w3.n, "parity_failures": fails}
    del d_buf, d_off, d_len, d_out, d_ok
    return leg, fails + (0 if all_ok else 1)


def config_c0_native():
    """configs[0] in the default line: one QP's 64 x 4156-B RDMA WRITE per
    message, compute + write_trailer then verify + zero_trailer, from 1 and 3 NATIVE threads (the
    emulator's send, packet-handler and receive threads are Rust, not Python: scripts/_build/msg_probe,
    C++) through the submission ring, pinned message buffers, ~0.5 s.  None when the probe is not
    built."""
    import icrc_amd

    probe = os.path.join(ROOT, "scripts", "_build", "msg_probe")
    if not os.path.exists(probe):
        return None
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(icrc_amd.LIB_PATH), MSG_PROBE_PATH="ring",
               MSG_PROBE_KINDS="pinned")
    try:
        r = subprocess.run([probe, "6000", "1", "3"], capture_output=True, text=True, timeout=60, env=env)
        rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    except (subprocess.TimeoutExpired, ValueError) as e:
        return {"error": f"msg_probe: {e}"}
    runs = [x for x in rows if "threads" in x]
    stats = next((x for x in rows if "ring_jobs" in x), {})
    if r.returncode != 0 or len(runs) != 2:
        return {"error": f"msg_probe exit {r.returncode}", "stderr": r.stderr[-400:]}
    one, three = runs
    return {"workload": "configs[0]: 64 x 4156-B RDMA WRITE per message in pinned host memory, compute + "
                        "write_trailer then verify + zero_trailer, native threads through the submission ring",
            "messages_per_s_1_thread": one["messages_per_s"], "p50_us_1_thread": one["message_p50_us"],
            "p99_us_1_thread": one["message_p99_us"],
            "messages_per_s_3_threads": three["messages_per_s"], "p50_us_3_threads": three["message_p50_us"],
            "p99_us_3_threads": three["message_p99_us"],
            "GiB/s_3_threads": round(three["messages_per_s"] * 64 * 4156 / GIB, 2),
            "calls_per_thread": 6000, "bad": one["bad"] + three["bad"],
            "ring": {k: stats.get(k) for k in ("ring_jobs", "ring_launches", "ring_relaunches", "ring_timeouts")}}


def per_rank_fields(rows):
    """Rank-0 summary of every rank's [kernel ms, device ordinal, wall ms per step, loads-only ms]
    (shard.gather_floats): a slow GPU or an imbalance shows here, not only in the max."""
    kms = [r[0] for r in rows]
    return {
        "kernel_ms": [round(x, 4) for x in kms],
        "device": [int(r[1]) for r in rows],
        "wall_ms_per_step": [round(r[2], 4) for r in rows],
        "loads_only_ms": [round(r[3], 4) for r in rows],
        "kernel_ms_min": round(min(kms), 4),
        "kernel_ms_max": round(max(kms), 4),
    }


def check_sample(orc, d_buf, d_out, n: int, L: int, k: int, rank: int, inject_rank: int):
    """Rank-local parity: the first and last k packets of this rank's batch against the CPU
    restatement.  Returns (mismatches, packets checked)."""
    spans = [(0, min(n, k))]
    if n > k:
        spans.append((max(k, n - k), n))
    fails = checked = 0
    got_all = d_out.cpu().numpy().view(np.uint32)
    for a, b in spans:
        host = d_buf[a * L: b * L].cpu().numpy()
        off = np.arange(b - a, dtype=np.uint64) * np.uint64(L)
        want = orc.compute_icrc_batch(host, off, np.full(b - a, L, np.uint32))
        got = got_all[a:b].copy()
        if rank == inject_rank:
            got[0] ^= 1
        fails += int(np.count_nonzero(got != want))
        checked += b - a
    return fails, checked


PMC_TRAFFIC_FILE = "r06_pmc_traffic.json"
PMC_C2_FILE = "r06_pmc_c2_traffic.json"
# the sources the C1 kernel is built from: a traffic summary taken on another build is not this one's
KERNEL_SOURCES = ("icrc_kernels.hip", "icrc_device.h", "icrc_long.h", "icrc_internal.h", "icrc_tables.cpp")
# ... and the configs[2] kernel (the hybrid launch: oct + long-packet workgroups)
C2_SOURCES = ("icrc_oct.hip", "icrc_device.h", "icrc_long.h", "icrc_internal.h", "icrc_tables.cpp")


def kernel_source_hash(names=KERNEL_SOURCES) -> str:
    """sha256 (16 hex digits) over a kernel's sources as shipped in this tree, comments and
    blank lines removed (a comment edit does not orphan a traffic record; any code edit does)."""
    import hashlib
    import re

    h = hashlib.sha256()
    for name in names:
        with open(os.path.join(ROOT, "open-rdma-driver_amd", "csrc", name), "r", encoding="utf-8") as f:
            text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        code = [ln.split("//", 1)[0].rstrip() for ln in text.splitlines()]
        h.update(name.encode() + b"\0" + "\n".join(ln for ln in code if ln).encode())
    return h.hexdigest()[:16]
LOADS_ONLY_VARIANT = 19  # A/B library: icrc_batch_kernel<.., S = 2, D = 1, loads only>, the default ring without the CRC


def pmc_record(fname: str, sources, n: int, L):
    """A committed PMC traffic record (profiles/<fname>) when it was taken on this exact workload
    (n packets; L bytes each, or None for a ragged batch) AND this build of its kernel's sources
    (kernel_source_hash); otherwise None."""
    path = os.path.join(ROOT, "profiles", fname)
    try:
        with open(path) as f:
            tr = json.load(f)
    except (OSError, ValueError):
        return None
    if tr.get("packets") != n or (L is not None and tr.get("packet_bytes") != L):
        return None
    if tr.get("source_hash") != kernel_source_hash(sources):  # profiled on another build of the kernel
        log(f"bench.py: profiles/{fname} is of kernel sources {tr.get('source_hash')}, this tree is "
            f"{kernel_source_hash(sources)}: its traffic is left null")
        return None
    return tr


def pmc_traffic(n: int, L: int):
    """roofline.traffic: HBM bytes per launch of the ICRC kernel from rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE in separate runs of this same bench command, FETCH_SIZE corrected
    by the membench calibration; scripts/gpu_check.sh PMC=1 -> scripts/pmc_summary.py).  A bench
    process cannot read its own counters, so the committed summary is used when it was taken on
    this exact workload AND this build of the kernel (kernel_source_hash); otherwise None."""
    return pmc_record(PMC_TRAFFIC_FILE, KERNEL_SOURCES, n, L)


def _timed_loop(fn, budget: float):
    """Repeat fn() (returns (seconds, ...)) until `budget` seconds of measured time."""
    secs, passes, last = 0.0, 0, None
    while secs < budget or passes == 0:
        last = fn()
        secs += last[0]
        passes += 1
    return secs, passes, last


def cpu_baseline(orc, host, L: int, d_out, args):
    """cpu_baseline: compute_icrc with the crc32fast-1.4.2-equivalent PCLMULQDQ core on one core
    over a bounded sample of the same packets.  cpu_context, beside it: the same on
    every core of this job's CPU share (the box caps a job at 16; os.cpu_count() reports the whole
    machine); the verify leg (is_icrc_valid, with and without the trailer zeroing); the emulator's
    per-packet send path (8 KiB alloc + memset, copy in, CRC, copy out: net/util.rs:172-186,
    packet_processor.rs:210-265); and configs[0] as stated — one QP's 64 x 4156-B WRITE (256 KiB,
    FIRST + 62 MIDDLE + LAST), compute on send then verify with zeroing on receive, per packet."""
    cs = host.size // L
    got = d_out[:cs].cpu().numpy().view(np.uint32)
    secs, passes, last = _timed_loop(lambda: orc.fast_icrc_strided_timed(host, L, L, cs, threads=1), args.cpu_seconds)
    cpu_ok = bool(np.array_equal(last[1], got))
    base = {
        "value": round(cs * L * passes / secs / GIB, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{cs} x {L}-B packets of the same batch, {passes} passes, {secs:.1f} s; compute_icrc "
                  f"with a crc32fast-1.4.2-equivalent PCLMULQDQ core (oracle/icrc_fast.c); matches GPU: {cpu_ok}",
    }
    threads = max(1, min(16, os.cpu_count() or 1))
    budget = args.cpu_seconds / 5
    ctx = {}

    def rate(fn, nbytes):
        s, p, last = _timed_loop(fn, budget)
        return round(nbytes * p / s / GIB, 3), round(s, 2), last

    g, s, _ = rate(lambda: orc.fast_icrc_strided_timed(host, L, L, cs, threads=threads), cs * L)
    ctx["compute_all_cores"] = {"GiB/s": g, "cores": threads, "seconds": s}
    vbuf = host.copy()
    orc_out = orc.fast_icrc_strided_timed(host, L, L, cs, threads=threads)[1]
    vbuf.reshape(cs, L)[:, L - 4:] = orc_out.view(np.uint8).reshape(cs, 4)  # trailers written
    for name, th in (("verify_1_core", 1), ("verify_all_cores", threads)):
        g, s, last = rate(lambda th=th: orc.fast_verify_strided_timed(vbuf, L, L, cs, threads=th, zero=False), cs * L)
        ctx[name] = {"GiB/s": g, "cores": th, "seconds": s, "all_ok": bool(last[1].all())}
    zb = vbuf.copy()
    s0, ok0 = orc.fast_verify_strided_timed(zb, L, L, cs, threads=1, zero=True)
    ctx["verify_zero_trailer_1_core"] = {"GiB/s": round(cs * L / s0 / GIB, 3), "cores": 1, "seconds": round(s0, 2),
                                         "all_ok": bool(ok0.all()), "note": "one pass (the zeroing is destructive)"}
    g, s, _ = rate(lambda: orc.fast_emulator_path_timed(host, L, L, cs), cs * L)
    ctx["emulator_send_path_1_core"] = {"GiB/s": g, "cores": 1, "seconds": s}
    c0buf, c0off, c0len = orc.synth_write(256 << 10, 4096, local_va=0x7F7E8EE00000, remote_va=0x7F7E8FC00000,
                                          rkey=0x2000003, dqpn=2, psn0=0, msn=0, dst_ip=0xC0A80003,
                                          payload_key=0xC0)
    c0bytes = int(c0len.astype(np.uint64).sum())
    for name, th in (("c0_roundtrip_1_core", 1), ("c0_roundtrip_all_cores", threads)):
        reps = 50
        s, p, last = _timed_loop(lambda th=th: orc.fast_c0_roundtrip_timed(c0buf, c0off, c0len, threads=th, reps=reps),
                                 budget)
        ctx[name] = {"GiB/s": round(c0bytes * reps * th * p / s / GIB, 3), "cores": th, "seconds": round(s, 2),
                     "packets_per_message": int(c0len.size), "failed_verifies": last[1],
                     "what": "configs[0]: 64 x 4156-B WRITE, emulator send path + is_icrc_valid (zeroing) per packet"}
    return base, ctx


# ---- secondary configs -----------------------------------------------------------------------
def dev(a: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def extra_measurements(eng, stream, args, world):
    """Secondary configs: verify pass, trailer store / zeroing (the reference's own store
    semantics), mixed MTU (configs[2]), 16 MiB round trip (configs[3]), the fused send /
    receive kernels and the host-resident (PCIe) rate."""
    import torch

    from icrc_amd import workloads

    ex = {}
    n = args.packets
    w = workloads.write_middle_stream(n, args.pmtu)
    L = int(w.lens[0])
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")

    def frac(ms, nbytes):
        return round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    # PacketWriter::write stores the trailer (packet_processor.rs:263): compute + write_trailer
    _, kms = time_kernel(lambda: eng.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), True, stream),
                         args.steps, args.warmup, world)
    ex["compute_c1_write_trailer"] = {"kernel_ms": round(kms, 4), "GiB/s": round(n * L / (kms * 1e-3) / GIB, 1),
                                      "frac_of_peak": frac(kms, n * L)}
    # verify over the C1 batch with trailers written
    _, kms = time_kernel(lambda: eng.verify_strided(d_buf.data_ptr(), L, L, n, d_ok.data_ptr(), False, stream),
                         args.steps, args.warmup, world)
    ex["verify_c1"] = {"GiB/s": round(n * L / (kms * 1e-3) / GIB, 1), "kernel_ms": round(kms, 4),
                       "frac_of_peak": frac(kms, n * L), "all_ok": bool((d_ok == 1).all().item())}
    # is_icrc_valid zeroes the trailer (packet_processor.rs:350): the first pass sees the real
    # trailers (checked), later passes compare against zeros — the same work and traffic
    eng.verify_strided(d_buf.data_ptr(), L, L, n, d_ok.data_ptr(), True, stream)
    torch.cuda.synchronize()
    first_ok = bool((d_ok == 1).all().item())
    zeroed = bool((d_buf.view(n, L)[:, L - 4:] == 0).all().item())
    _, kms = time_kernel(lambda: eng.verify_strided(d_buf.data_ptr(), L, L, n, d_ok.data_ptr(), True, stream),
                         args.steps, args.warmup, world)
    ex["verify_c1_zero_trailer"] = {"kernel_ms": round(kms, 4), "GiB/s": round(n * L / (kms * 1e-3) / GIB, 1),
                                    "frac_of_peak": frac(kms, n * L), "first_pass_all_ok": first_ok,
                                    "trailers_zeroed": zeroed}
    del d_buf, d_out, d_ok

    # C1 at the padded stride (packed 4156 and padded 4224 both measured): every
    # packet 64-byte aligned, the same 4156 bytes each
    wp = workloads.write_middle_stream(n, args.pmtu, stride=4224)
    d_buf = workloads.synthesize(eng, wp, stream=stream)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    _, kms = time_kernel(lambda: eng.compute_strided(d_buf.data_ptr(), 4224, L, n, d_out.data_ptr(), False, stream),
                         args.steps, args.warmup, world)
    ex["compute_c1_stride_4224"] = {"kernel_ms": round(kms, 4), "GiB/s": round(n * L / (kms * 1e-3) / GIB, 1),
                                    "frac_of_peak": frac(kms, n * L)}
    del d_buf, d_out

    # C1's packets as a ragged batch (offset / length arrays, the default hybrid dispatch): what a
    # driver's packet buffers hand over; the arrays' 12 bytes per packet are not counted
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_off, d_len = dev(w.off), dev(w.lens)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    _, kms = time_kernel(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                                   d_out.data_ptr(), False, 0, stream),
                         args.steps, args.warmup, world)
    ex["compute_c1_ragged"] = {"kernel_ms": round(kms, 4), "GiB/s": round(n * L / (kms * 1e-3) / GIB, 1),
                               "frac_of_peak": frac(kms, n * L)}
    del d_buf, d_out, d_off, d_len

    # mixed MTU
    wm = workloads.mixed_mtu_stream(4 << 20)
    d_buf = workloads.synthesize(eng, wm, stream=stream)
    d_off, d_len = dev(wm.off), dev(wm.lens)
    d_out = torch.zeros(wm.n, dtype=torch.int32, device="cuda")
    _, kms = time_kernel(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n,
                                                   d_out.data_ptr(), False, 0, stream),
                         args.steps, args.warmup, world)
    tot = int(wm.lens.astype(np.uint64).sum())
    ex["mixed_mtu_c2"] = {"packets": wm.n, "bytes": tot, "GiB/s": round(tot / (kms * 1e-3) / GIB, 1),
                          "kernel_ms": round(kms, 4), "frac_of_peak": frac(kms, tot)}
    del d_buf, d_out, d_off, d_len

    # 16 MiB WRITE round trip: compute(send, write trailer) + verify(recv, zero trailer)
    w3 = workloads.write_message(16 << 20, 4096)
    d_buf = workloads.synthesize(eng, w3, stream=stream)
    d_off, d_len = dev(w3.off), dev(w3.lens)
    d_out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    d_ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def rt():
        eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_out.data_ptr(), True, 0, stream)
        eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_ok.data_ptr(), True, 0, stream)

    _, kms = time_kernel(rt, args.steps, args.warmup, world)
    tot3 = int(w3.lens.astype(np.uint64).sum())
    ex["roundtrip_16MiB_c3"] = {"packets": w3.n, "ms_per_roundtrip": round(kms, 4),
                                "GiB/s_per_direction": round(2 * tot3 / (kms * 1e-3) / GIB, 1),
                                "all_ok": bool((d_ok == 1).all().item())}
    del d_buf, d_off, d_len, d_out, d_ok

    ex.update(fused_send_receive(eng, stream, args, world))
    ex.update(receive_short(eng, stream, args, world))
    ex.update(host_resident(eng, stream, args))
    ex.update(host_message_c0(eng, stream, args))
    return ex


def fused_send_receive(eng, stream, args, world):
    """§8f rows 1-3 at C1 scale: the fused send packetizer turning 192 x 16 MiB RDMA WRITE
    messages (786 K x 4156-B packets) into wire packets with trailers, then the fused receive
    (verify + strip + parse) over the same wire buffer.  Algorithmic HBM bytes per packet:
    send = 4096 payload read + 4156 wire write + 8 result; receive = 4156 read + 72 descriptor
    + 1 ok byte written."""
    import torch

    import icrc_amd

    out = {}
    nmsg, msg_bytes, pmtu = max(1, min(args.packets, 3 << 18) // 4096), 16 << 20, 4096  # 3 GiB of payload
    specs = [dict(local_va=0x7F0000000000 + i * msg_bytes, remote_va=0x7E0000000000 + i * msg_bytes,
                  payload_offset=i * msg_bytes, total_len=msg_bytes, pmtu=pmtu, rkey=0x2000003, dqpn=2 + i,
                  psn=0, msn=i & 0xFFFF, dst_ip=0xC0A80003, kind=0) for i in range(nmsg)]
    msgs = icrc_amd.write_messages(specs, slot_stride=28 + 28 + pmtu + 4)
    npk = int(msgs["npackets"].sum())
    src_bytes = nmsg * msg_bytes
    wire_bytes = npk * (28 + 28 + pmtu + 4)
    g = torch.Generator(device="cuda").manual_seed(5)
    d_src = torch.empty(src_bytes, dtype=torch.uint8, device="cuda")
    for c0 in range(0, src_bytes, 1 << 30):  # < 2^31 elements per torch kernel
        c1 = min(src_bytes, c0 + (1 << 30))
        d_src[c0:c1] = torch.randint(0, 256, (c1 - c0,), dtype=torch.uint8, device="cuda", generator=g)
    torch.cuda.synchronize()
    d_msgs = dev(msgs.view(np.uint8))
    d_wire = torch.empty(wire_bytes, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")

    def send():
        eng.packetize(d_src.data_ptr(), src_bytes, d_msgs.data_ptr(), nmsg, npk, d_wire.data_ptr(), wire_bytes,
                      d_len.data_ptr(), d_icrc.data_ptr(), stream)

    _, kms = time_kernel(send, args.steps, args.warmup, world)
    torch.cuda.synchronize()
    lens_ok = bool((d_len == 28 + 28 + pmtu + 4).all().item())
    log(f"packetize: {npk} packets, {kms:.4f} ms, lengths ok {lens_ok}")
    alg = npk * (4096 + 4156 + 8)
    out["packetize_send"] = {"packets": npk, "kernel_ms": round(kms, 4),
                             "wire_GiB/s": round(wire_bytes / (kms * 1e-3) / GIB, 1),
                             "hbm_GB/s": round(alg / (kms * 1e-3) / 1e9, 1),
                             "frac_of_peak": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "lengths_ok": lens_ok}
    if not lens_ok:
        return out
    # same-box denominator: a device-to-device copy of the payload bytes (hipMemcpyAsync through
    # torch) into the wire buffer, then the packets are rebuilt for the receive leg
    _, cms = time_kernel(lambda: d_wire[:src_bytes].copy_(d_src), args.steps, args.warmup, world)
    send()
    torch.cuda.synchronize()
    out["packetize_send"]["copy_reference"] = {
        "what": "d2d copy of the same payload bytes (hipMemcpyAsync), same box, timed like the kernel",
        "ms": round(cms, 4), "hbm_GB/s": round(2 * src_bytes / (cms * 1e-3) / 1e9, 1),
        "packetize_rate_vs_copy_rate": round((alg / kms) / (2 * src_bytes / cms), 4)}
    del d_src
    d_off = torch.arange(npk, dtype=torch.int64, device="cuda") * (28 + 28 + pmtu + 4)
    d_desc = torch.empty(npk * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(npk, dtype=torch.uint8, device="cuda")

    def recv():
        eng.rx_parse(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_desc.data_ptr(), d_ok.data_ptr(),
                     stream=stream)

    _, kms = time_kernel(recv, args.steps, args.warmup, world)
    alg = npk * (4156 + 72 + 1)
    desc = d_desc[: 64 * 72].cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    out["rx_verify_parse"] = {"packets": npk, "kernel_ms": round(kms, 4),
                              "GiB/s": round(wire_bytes / (kms * 1e-3) / GIB, 1),
                              "hbm_GB/s": round(alg / (kms * 1e-3) / 1e9, 1),
                              "frac_of_peak": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "all_ok": bool((d_ok == 1).all().item()),
                              "payload_len_ok": bool(np.all(desc["payload_len"] == pmtu))}
    return out


def rx_leg(eng, stream, args, world, w, ragged, orc=None, sample=0):
    """One receive leg: w's packets synthesised, their trailers written by a compute pass, then
    icrc_rx_parse_device (verify + strip + parse) timed like the headline.  sample > 0: the first and
    last `sample` packets' descriptors and ok bytes against the oracle's rx_parse (the checker)."""
    import torch

    import icrc_amd
    from icrc_amd import workloads

    desc_b = icrc_amd.RX_DESC_DTYPE.itemsize
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_off, d_len = dev(w.off), dev(w.lens)
    d_tmp = torch.zeros(w.n, dtype=torch.int32, device="cuda")
    eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_tmp.data_ptr(), True, 0, stream)
    torch.cuda.synchronize()
    del d_tmp
    d_desc = torch.empty(w.n * desc_b, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
    L = int(w.lens[0])
    if ragged:
        fn = lambda: eng.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, d_desc.data_ptr(),
                                  d_ok.data_ptr(), stream=stream)
    else:
        fn = lambda: eng.rx_parse(d_buf.data_ptr(), 0, 0, w.n, d_desc.data_ptr(), d_ok.data_ptr(),
                                  stride=L, length=L, stream=stream)
    _, kms = time_kernel(fn, min(args.steps, 20), min(args.warmup, 5), world)
    tot = int(w.lens.astype(np.uint64).sum())
    alg = tot + w.n * (desc_b + 1)
    desc = d_desc[: 64 * desc_b].cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
    res = {"packets": w.n, "packet_bytes": tot, "kernel_ms": round(kms, 4),
           "hbm_GB/s": round(alg / (kms * 1e-3) / 1e9, 1), "frac_of_peak": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "all_ok": bool((d_ok == 1).all().item()), "first_desc_payload_len": int(desc["payload_len"][0])}
    if sample and orc is not None:
        got_all = d_desc.view(w.n, desc_b)
        fails = 0
        for a, b in ((0, min(sample, w.n)), (max(0, w.n - sample), w.n)):
            lo, hi = int(w.off[a]), int(w.off[b - 1]) + int(w.lens[b - 1])
            host = d_buf[lo:hi].cpu().numpy()
            want = orc.rx_parse(host, (w.off[a:b] - np.uint64(lo)).astype(np.uint64), w.lens[a:b])
            got = got_all[a:b].cpu().numpy().reshape(-1).view(icrc_amd.RX_DESC_DTYPE).copy()
            # the oracle parsed the sample from offset 0 (payload_offset is 0 on a packet that failed to parse)
            got["payload_offset"] = np.where(got["status"] == 0, got["payload_offset"] - np.uint64(lo),
                                             got["payload_offset"])
            for f in want.dtype.names:
                if f != "_pad":
                    fails += int(np.count_nonzero(got[f] != want[f]))
            fails += int(np.count_nonzero(d_ok[a:b].cpu().numpy() != want["icrc_ok"]))
        res["parity_checked"] = 2 * min(sample, w.n)
        res["parity_failures"] = fails
    del d_buf, d_off, d_len, d_desc, d_ok
    torch.cuda.empty_cache()
    return res


def config_c2_rx(eng, stream, args, world, orc):
    """configs[2]'s batch through the receive parse: mixed_mtu_stream(4 Mi) with
    its trailers written, icrc_rx_parse_device on the default ragged dispatch; algorithmic bytes =
    packets read + a 72-byte descriptor and an ok byte written per packet; 4096 descriptors (both ends)
    against the oracle.  Returns (leg, mismatches)."""
    from icrc_amd import workloads

    r = rx_leg(eng, stream, args, world, workloads.mixed_mtu_stream(4 << 20), True, orc, 2048)
    leg = {"workload": "configs[2] received: 4 Mi mixed-MTU packets, icrc_rx_parse_device (verify + strip + parse "
                       "into 72-byte descriptors), ragged arrays",
           "packets": r["packets"], "kernel_ms": r["kernel_ms"], "hbm_GB/s": r["hbm_GB/s"], "frac": r["frac_of_peak"],
           "all_ok": r["all_ok"], "parity_checked": r["parity_checked"], "parity_failures": r["parity_failures"]}
    return leg, r["parity_failures"] + (0 if r["all_ok"] else 1)


def receive_short(eng, stream, args, world):
    """§8f row 3 at the emulator's receive shapes: icrc_rx_parse_device (verify + strip + parse)
    over configs[2]'s mixed-MTU batch with its trailers written (`rx_verify_parse_c2`, with 4096
    descriptors checked against the oracle), and over 4 Mi 316-byte packets (the 256-B MTU class) as
    a ragged batch and as a strided one.  Algorithmic HBM bytes per packet: the packet read + a
    72-byte descriptor + an ok byte written."""
    import oracle as orc
    from icrc_amd import workloads

    out = {}
    out["rx_verify_parse_c2"] = rx_leg(eng, stream, args, world, workloads.mixed_mtu_stream(4 << 20), True, orc, 2048)
    w316 = workloads.write_middle_stream(4 << 20, 256)
    out["rx_verify_parse_316_ragged"] = rx_leg(eng, stream, args, world, w316, True, orc, 2048)
    out["rx_verify_parse_316_strided"] = rx_leg(eng, stream, args, world, w316, False, orc, 2048)
    return out


def host_resident(eng, stream, args):
    """Packets in host memory (pinned and pageable) -> H2D -> kernel -> ICRCs back (PCIe bound;
    never the headline value)."""
    import torch

    from icrc_amd import workloads

    ex = {}
    nh = min(args.packets, 1 << 18)
    wh = workloads.write_middle_stream(nh, args.pmtu)
    Lh = int(wh.lens[0])
    d_buf = workloads.synthesize(eng, wh, stream=stream)
    h_buf = torch.empty(wh.total_bytes, dtype=torch.uint8, pin_memory=True)
    h_buf.copy_(d_buf)
    torch.cuda.synchronize()
    d_ref = torch.zeros(wh.n, dtype=torch.int32, device="cuda")
    eng.compute_strided(d_buf.data_ptr(), Lh, Lh, wh.n, d_ref.data_ptr(), False, stream)
    torch.cuda.synchronize()
    ref = d_ref.cpu().numpy().view(np.uint32)
    del d_buf
    h_np = h_buf.numpy()
    p_np = h_np.copy()  # pageable copy of the same packets
    reps = max(3, args.steps // 4)
    got = None
    for name, arr in (("pinned", h_np), ("pageable", p_np)):
        eng.compute_batch_host(arr, wh.off, wh.lens)  # warm (allocates the stages)
        t0 = time.perf_counter()
        for _ in range(reps):
            got = eng.compute_batch_host(arr, wh.off, wh.lens)
        secs = (time.perf_counter() - t0) / reps
        ex[f"host_resident_{name}"] = {
            "packets": nh, "GiB/s": round(nh * Lh / secs / GIB, 2), "ms": round(secs * 1e3, 3),
            "note": "icrc_compute_batch_ex: packets in host memory -> H2D (64 MiB chunks, 2 streams "
                    "overlapping copy and kernel) -> ICRCs back to host; PCIe Gen5 x16 bound"}
    ex["host_resident_results_match_device"] = bool(np.array_equal(got, ref))
    return ex


def host_message_c0(eng, stream, args):
    """configs[0]-shaped messages through the host-resident drop-ins, per message: one QP's 256 KiB
    RDMA WRITE (64 x 4156-B packets, FIRST + 62 MIDDLE + LAST) in host memory, the send side's
    icrc_compute_batch(write_trailer=1) (PacketWriter::write stores the ICRC, packet_processor.rs:
    260-263) then the receive side's icrc_verify_batch(zero_trailer=1) (is_icrc_valid,
    packet_processor.rs:341-353; udp_agent.rs:99) — what the emulator's send and receive threads
    would call per message (queues/send/operations/write.rs:31-96).  Pinned and pageable buffers,
    from 1 and 3 threads (each thread its own message buffer, the default engine shared, as the
    reference's three callers would).  p50 / p99 microseconds per message (compute + verify)."""
    import threading

    import torch

    import icrc_amd
    from icrc_amd import workloads

    w = workloads.write_message(256 << 10, 4096)
    d_buf = workloads.synthesize(eng, w, stream=stream)
    torch.cuda.synchronize()
    src = d_buf.cpu().numpy()
    off, lens = np.ascontiguousarray(w.off, np.uint64), np.ascontiguousarray(w.lens, np.uint32)
    nbytes = int(lens.astype(np.uint64).sum())
    reps = max(1000, args.steps * 4)
    out = {}
    for kind in ("pinned", "pageable"):
        for nth in (1, 3):
            bufs = []
            for _ in range(nth):
                if kind == "pinned":
                    t = torch.empty(src.size, dtype=torch.uint8, pin_memory=True)
                    b = t.numpy()
                    b[:] = src
                    bufs.append((t, b))
                else:
                    bufs.append((None, src.copy()))
            lat = [[] for _ in range(nth)]
            bad = [0] * nth
            ends = [0.0] * nth
            start = [0.0]
            # warm-up calls (first touch of the buffer, the ring's launch) outside the timed region:
            # every thread warms, then all are released together; messages/s = the timed messages
            # over (last thread's end - release).  (Round 4 counted thread start and the warm-up
            # calls in the rate: the 1-thread pinned case, first in the sequence, read half its p50.)
            gate = threading.Barrier(nth, action=lambda: start.__setitem__(0, time.perf_counter()))

            def worker(k):
                b = bufs[k][1]
                for i in range(reps + 20):
                    if i == 20:
                        gate.wait()
                    t0 = time.perf_counter_ns()
                    icrc_amd.compute_icrc_batch(b, off, lens, write_trailer=True)
                    ok = icrc_amd.verify_icrc_batch(b, off, lens, zero_trailer=True)
                    t1 = time.perf_counter_ns()
                    if i >= 20:
                        lat[k].append((t1 - t0) / 1e3)
                    bad[k] += int(np.count_nonzero(ok != 1))
                ends[k] = time.perf_counter()

            ths = [threading.Thread(target=worker, args=(k,)) for k in range(nth)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            secs = max(ends) - start[0]
            allv = np.concatenate([np.asarray(x) for x in lat])
            out[f"c0_message_{kind}_{nth}_thread"] = {
                "p50_us": round(float(np.percentile(allv, 50)), 1), "p99_us": round(float(np.percentile(allv, 99)), 1),
                "mean_us": round(float(np.mean(allv)), 1),
                "messages_per_s": round(nth * reps / secs, 1),
                "GiB/s": round(nth * reps * nbytes / secs / GIB, 3),
                "failed_verifies": int(sum(bad)), "packets_per_message": int(w.n), "message_bytes": nbytes}
    out["c0_message_note"] = ("per message: icrc_compute_batch(write_trailer=1) + icrc_verify_batch(zero_trailer=1) on "
                              "a 64 x 4156-B WRITE in host memory; compare cpu_context.c0_roundtrip_1_core")
    # The same calls from native threads (scripts/_build/msg_probe, C++: the reference's callers are
    # Rust threads; Python threads serialise on the GIL around every ctypes call), 1 and 3 threads:
    # through the submission ring (the default host path) and one launch per call (ICRC_HOST_LAUNCH).
    probe = os.path.join(ROOT, "scripts", "_build", "msg_probe")
    if os.path.exists(probe):
        for key, path in (("c0_message_native", "ring"), ("c0_message_native_launch", "launch")):
            env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(icrc_amd.LIB_PATH), MSG_PROBE_PATH=path)
            try:
                r = subprocess.run([probe, "1000", "1", "3"], capture_output=True, text=True, timeout=180, env=env)
                out[key] = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
            except (subprocess.TimeoutExpired, ValueError) as e:
                out[key] = f"msg_probe failed: {e}"
    return out


# ---- CPU stub (tests): the N>1 plumbing without GPUs -------------------------------------------
def run_cpu_stub(args, rank: int, world: int) -> int:
    import zlib

    import torch.distributed as dist

    from icrc_amd import shard

    if world > 1:
        dist.init_process_group("gloo", timeout=_dist_timeout(args))
    if rank == args.stall_rank:  # tests: a rank that never reaches the first barrier
        time.sleep(3600)
    L = 28 + 28 + args.pmtu + 4
    if args.scaling == "weak":  # one stream per rank
        lo, hi, key = 0, args.packets, 0x5EED5EED + rank
    else:  # one stream, sliced: strong-scaling shards are exactly its packet ranges
        (lo, hi), key = shard.shard_range(args.packets, rank, world), 0x5EED5EED
    n = hi - lo
    buf = np.random.default_rng(key).integers(0, 256, hi * L, dtype=np.uint8)[lo * L:]
    out = np.zeros(n, dtype=np.uint32)

    def step():  # CPU stand-in for the kernel launch (NOT the ICRC)
        for i in range(n):
            out[i] = zlib.crc32(buf[i * L:(i + 1) * L])

    wall, _ = time_steps(step, args.steps, args.warmup, world, lambda: None, dist.barrier if world > 1 else None)
    want = np.array([zlib.crc32(buf[i * L:(i + 1) * L]) for i in range(n)], dtype=np.uint32)
    got = out.copy()
    if rank == args.inject_fault_rank and n:
        got[0] ^= 1
    fails = int(np.count_nonzero(got != want))
    agg = shard.aggregate(n * L * args.steps, wall, fails)
    per_rank = shard.gather_floats([wall / args.steps * 1e3, rank, wall / args.steps * 1e3, 0.0])
    if rank == 0:
        print(json.dumps({
            "metric": METRIC + " [cpu-stub: plumbing test, not the ICRC]", "value": round(agg.gib_per_s, 6),
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(agg.seconds / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u8", "data": "synthetic (cpu stub)",
            "config": {"workload": "cpu-stub", "packets_per_gpu": n, "packet_bytes": L,
                       "bytes_total_per_step": agg.total_bytes // args.steps,
                       "packets_total_per_step": agg.total_bytes // args.steps // L,
                       "parallelism": f"shard-per-rank x{world} (gloo)"},
            "parity_sample": {"failures_all_ranks": agg.failures},
            "per_rank": per_rank_fields(per_rank),
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 1 if agg.failures else 0


if __name__ == "__main__":
    sys.exit(main())
