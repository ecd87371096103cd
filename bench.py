#!/usr/bin/env python3
"""bench.py — device-resident ICRC throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1 Mi x 4 KiB-MTU RDMA WRITE_MIDDLE packets (L = 4156 B:
IPv4 20 + UDP 8 + BTH 12 + RETH 16 + 4096 payload + ICRC 4), synthesised on the device with
the reference's PacketWriter field layout; one "step" = one ICRC-compute pass (kernel launch)
over the whole batch, inputs resident in HBM, ICRCs written to an HBM array.

Multi-GPU (--gpus N via torch.distributed.run): one process per GPU, each with its own
independent QP stream of 1 Mi packets (configs[4], weak scaling, no collective on the
data path; the only collectives are the timing barrier and a max over ranks).

Prints ONE JSON line (rank 0).  value = whole-job GiB/s of packet bytes (sum of L, which
equals the algorithmic bytes: L-4 read + 4 written per packet).  roofline = the ICRC kernel's
achieved GB/s (HIP events on the launch stream) vs the 8.0 TB/s HBM3E peak.  cpu_baseline =
the CPU port of compute_icrc with a crc32fast-equivalent PCLMULQDQ core (oracle/icrc_fast.c),
rank 0 / N=1 only, on a bounded sample of the same packets.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def log(msg: str) -> None:
    print(msg, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU")
    ap.add_argument("--pmtu", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline time budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--extra", action="store_true",
                    help="also time verify, mixed-MTU, 16 MiB round trip and the host-resident path")
    return ap.parse_args()


PMC_TRAFFIC_FILE = "r01_pmc_traffic.json"


def pmc_traffic(n: int, L: int):
    """roofline.traffic: HBM bytes per launch of the ICRC kernel from rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE in separate runs of this same bench command, FETCH_SIZE corrected
    by the membench calibration; scripts/gpu_check.sh PMC=1 -> scripts/pmc_summary.py).  A bench
    process cannot read its own counters, so the committed summary is used when it was taken on
    this exact workload; otherwise None."""
    path = os.path.join(ROOT, "profiles", PMC_TRAFFIC_FILE)
    try:
        with open(path) as f:
            tr = json.load(f)
    except (OSError, ValueError):
        return None
    if tr.get("packets") != n or tr.get("packet_bytes") != L:
        return None
    return tr


def dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def time_kernel(fn, steps: int, warmup: int, world: int):
    """Warmup, barrier+sync, K timed launches (HIP events on the current stream), sync+barrier.
    Returns (wall seconds, max over ranks; kernel ms per launch from events)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    return wall, ev0.elapsed_time(ev1) / steps


def main() -> int:
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import icrc_amd
    from icrc_amd import workloads

    eng = icrc_amd.Engine(local)
    stream = torch.cuda.current_stream().cuda_stream

    # ---- C1 workload: one QP stream per rank (dqpn = 2 + rank, distinct payload seed) ----
    n = args.packets
    w = workloads.write_middle_stream(n, args.pmtu, dqpn=2 + rank, payload_key=0x5EED5EED + rank)
    L = int(w.lens[0])
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def step():
        eng.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), False, stream)

    wall, kms = time_kernel(step, args.steps, args.warmup, world)
    bytes_per_step = n * L
    value = world * bytes_per_step * args.steps / wall / GIB
    achieved = bytes_per_step / (kms * 1e-3) / 1e9

    result = {
        "metric": "device-resident ICRC GiB/s over 4 KiB-MTU packet batches; % of HBM-read roofline",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-synthesised RDMA WRITE_MIDDLE packets, splitmix64 payload)",
        "config": {
            "workload": "configs[1]: 1Mi x 4KiB-MTU packets per GPU, device-resident ICRC compute"
                        + (f" (configs[4]: {world} independent QP streams, one per GPU)" if world > 1 else ""),
            "packets_per_gpu": n,
            "packet_bytes": L,
            "pmtu": args.pmtu,
            "bytes_per_gpu_per_step": bytes_per_step,
            "parallelism": f"shard-per-gpu x{world} (no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "icrc_batch_kernel<kCompute>",
            "kernel_ms": round(kms, 4),
        },
    }
    tr = pmc_traffic(n, L)
    if tr is not None:
        result["roofline"]["traffic"] = tr["traffic_bytes"]
        result["roofline"]["traffic_source"] = (
            f"profiles/{PMC_TRAFFIC_FILE}: {tr['kernel']} HBM bytes per launch (FETCH_SIZE x "
            f"{tr['fetch_correction']} + WRITE_SIZE), {tr['ratio_to_algorithmic']}x the algorithmic bytes")

    # ---- CPU baseline: rank 0, N = 1 only ----
    parity = True
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle as orc  # the checker / CPU port: used only in this leg

        cs = min(n, 16384)  # 68 MB sample of the same packets
        host = d_buf[: cs * L].cpu().numpy()
        secs, passes = 0.0, 0
        cpu_out = None
        while secs < args.cpu_seconds or passes == 0:
            s, cpu_out = orc.fast_icrc_strided_timed(host, L, L, cs, threads=1)
            secs += s
            passes += 1
        cpu_ok = bool(np.array_equal(cpu_out, d_out[:cs].cpu().numpy().view(np.uint32)))
        parity = cpu_ok
        result["cpu_baseline"] = {
            "value": round(cs * L * passes / secs / GIB, 3),
            "unit": "GiB/s",
            "cores": 1,
            "kind": "port",
            "sample": f"{cs} x {L}-B packets of the same batch, {passes} passes, {secs:.1f} s; "
                      "compute_icrc with a crc32fast-1.4.2-equivalent PCLMULQDQ core "
                      f"(oracle/icrc_fast.c); matches GPU: {cpu_ok}",
        }
        result["parity_sample_ok"] = cpu_ok
        result["cpu_context"] = cpu_context(orc, host, L, cs, args.cpu_seconds / 4)

    if args.extra:
        result["extra"] = extra_measurements(eng, stream, args, world)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if parity else 1


def cpu_context(orc, host, L, cs, budget):
    """Beside the 1-core cpu_baseline: the same port on every core of this job's CPU
    share (the box caps a job at 16; os.cpu_count() reports the whole machine), and the emulator's
    per-packet send path around compute_icrc on one core (8 KiB vec alloc + memset, payload copy
    in, CRC, UDP-payload copy out: net/util.rs:172-186, packet_processor.rs:210-265)."""
    threads = max(1, min(16, os.cpu_count() or 1))
    out = {}
    for name, fn in (("all_cores", lambda: orc.fast_icrc_strided_timed(host, L, L, cs, threads=threads)),
                     ("emulator_path_1_core", lambda: orc.fast_emulator_path_timed(host, L, L, cs))):
        secs, passes = 0.0, 0
        while secs < budget or passes == 0:
            s, _ = fn()
            secs += s
            passes += 1
        out[name] = {"GiB/s": round(cs * L * passes / secs / GIB, 3),
                     "cores": threads if name == "all_cores" else 1, "seconds": round(secs, 2)}
    return out


def extra_measurements(eng, stream, args, world):
    """Secondary configs: verify pass, mixed MTU (configs[2]), 16 MiB round trip
    (configs[3]) and the host-resident (PCIe) rate."""
    import icrc_amd
    from icrc_amd import workloads

    ex = {}
    # verify over the C1 batch with trailers written
    n = args.packets
    w = workloads.write_middle_stream(n, args.pmtu)
    L = int(w.lens[0])
    d_buf = workloads.synthesize(eng, w, stream=stream)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), True, stream)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    wall, kms = time_kernel(lambda: eng.verify_strided(d_buf.data_ptr(), L, L, n, d_ok.data_ptr(), False, stream),
                            args.steps, args.warmup, world)
    ex["verify_c1"] = {"GiB/s": round(n * L / (kms * 1e-3) / GIB, 1), "kernel_ms": round(kms, 4),
                       "all_ok": bool((d_ok == 1).all().item())}
    del d_buf, d_out, d_ok

    # mixed MTU
    wm = workloads.mixed_mtu_stream(4 << 20)
    d_buf = workloads.synthesize(eng, wm, stream=stream)
    d_off, d_len = dev(wm.off), dev(wm.lens)
    d_out = torch.zeros(wm.n, dtype=torch.int32, device="cuda")
    wall, kms = time_kernel(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n,
                                                      d_out.data_ptr(), False, 0, stream),
                            args.steps, args.warmup, world)
    tot = int(wm.lens.astype(np.uint64).sum())
    ex["mixed_mtu_c2"] = {"packets": wm.n, "bytes": tot, "GiB/s": round(tot / (kms * 1e-3) / GIB, 1),
                          "kernel_ms": round(kms, 4)}
    del d_buf, d_out, d_off, d_len

    # 16 MiB WRITE round trip: compute(send, write trailer) + verify(recv)
    w3 = workloads.write_message(16 << 20, 4096)
    d_buf = workloads.synthesize(eng, w3, stream=stream)
    d_off, d_len = dev(w3.off), dev(w3.lens)
    d_out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    d_ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def rt():
        eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_out.data_ptr(), True, 0, stream)
        eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w3.n, d_ok.data_ptr(), False, 0, stream)

    wall, kms = time_kernel(rt, args.steps, args.warmup, world)
    tot3 = int(w3.lens.astype(np.uint64).sum())
    ex["roundtrip_16MiB_c3"] = {"packets": w3.n, "ms_per_roundtrip": round(kms, 4),
                                "GiB/s_per_direction": round(2 * tot3 / (kms * 1e-3) / GIB, 1),
                                "all_ok": bool((d_ok == 1).all().item())}
    del d_buf, d_off, d_len, d_out, d_ok

    ex.update(fused_send_receive(eng, stream, args, world))

    # host-resident: packets in pinned host memory -> H2D -> kernel -> D2H of ICRCs
    nh = min(args.packets, 1 << 18)
    wh = workloads.write_middle_stream(nh, args.pmtu)
    Lh = int(wh.lens[0])
    d_buf = workloads.synthesize(eng, wh, stream=stream)
    h_buf = torch.empty(wh.total_bytes, dtype=torch.uint8, pin_memory=True)
    h_buf.copy_(d_buf)
    del d_buf
    torch.cuda.synchronize()
    h_np = h_buf.numpy()
    p_np = h_np.copy()  # pageable copy of the same packets
    reps = max(3, args.steps // 4)
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
    ex["host_resident_results_match_device"] = bool(np.array_equal(got, host_icrc_ref(eng, h_np, wh, stream)))
    return ex


def fused_send_receive(eng, stream, args, world):
    """§8f rows 1-3 at C1 scale: the fused send packetizer turning 256 x 16 MiB RDMA WRITE
    messages (1 Mi x 4156-B packets) into wire packets with trailers, then the fused receive
    (verify + strip + parse) over the same wire buffer.  Algorithmic HBM bytes per packet:
    send = 4096 payload read + 4156 wire write + 8 result; receive = 4156 read + 72 descriptor
    + 1 ok byte written."""
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


def host_icrc_ref(eng, h_np, wh, stream):
    """Device-resident ICRCs of the same packets (to check the host-resident path)."""
    d = torch.from_numpy(h_np).cuda()
    L = int(wh.lens[0])
    d_out = torch.zeros(wh.n, dtype=torch.int32, device="cuda")
    eng.compute_strided(d.data_ptr(), L, L, wh.n, d_out.data_ptr(), False, stream)
    torch.cuda.synchronize()
    return d_out.cpu().numpy().view(np.uint32)


if __name__ == "__main__":
    sys.exit(main())
