#!/usr/bin/env python3
"""Time the fused send packetizer (icrc_write_packetize_device) on bench.py --extra's workload:
192 x 16 MiB RDMA WRITE messages -> 786 K x 4156-B wire packets.  Median of 5 x 10 launches,
HIP events on the launch stream.  Engine kernel variants (and wire slot strides) given on the
command line are timed alternately in the same process (A/B on one box).  One JSON line per
variant, stride and repetition.  Slot strides: 4156 (packed, what bench.py uses), 4224 (every
packet 128-byte aligned) and 8192 (the reference's own per-packet buffer, net/util.rs:173); the
algorithmic bytes per packet (4096 read + 4156 written + 8) are the same for every stride.  After
the packetizer, a device-to-device copy of the payload bytes (hipMemcpyAsync) is timed beside it.

usage: probe_send.py [reps] [variant ...] [--strides 4156,4224,8192]   (-1 = the default dispatch;
pkN = the default dispatch with ICRC_AB_PK=N, the A/B library's packetizer shapes and cuts)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402


def main():
    args = sys.argv[1:]
    strides = [56 + 4096 + 4]
    if "--strides" in args:
        k = args.index("--strides")
        strides = [int(x) for x in args[k + 1].split(",")]
        args = args[:k] + args[k + 2:]
    reps = int(args[0]) if args else 3
    nmsg, mb, pmtu = 192, 16 << 20, 4096
    specs = [dict(local_va=0x7F0000000000 + i * mb, remote_va=0x7E0000000000 + i * mb, payload_offset=i * mb,
                  total_len=mb, pmtu=pmtu, rkey=3, dqpn=2 + i, psn=0, msn=i, dst_ip=0xC0A80003, kind=0)
             for i in range(nmsg)]
    per_stride = {st: torch.from_numpy(icrc_amd.write_messages(specs, slot_stride=st).view(np.uint8)).cuda()
                  for st in strides}
    npk = int(icrc_amd.write_messages(specs, slot_stride=strides[0])["npackets"].sum())
    g = torch.Generator(device="cuda").manual_seed(5)
    src = torch.empty(nmsg * mb, dtype=torch.uint8, device="cuda")
    for c0 in range(0, src.numel(), 1 << 30):
        c1 = min(src.numel(), c0 + (1 << 30))
        src[c0:c1] = torch.randint(0, 256, (c1 - c0,), dtype=torch.uint8, device="cuda", generator=g)
    wire = torch.zeros(npk * max(strides), dtype=torch.uint8, device="cuda")
    ln = torch.zeros(npk, dtype=torch.int32, device="cuda")
    ic = torch.zeros(npk, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    builds = []
    for x in args[1:] or ["-1"]:
        eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())  # A/B library: diagnostic variants
        eng.set_variant(-1 if x.startswith("pk") else int(x))
        builds.append((x, eng))
    alg = npk * (4096 + 4156 + 8)
    ref = {}
    for r in range(reps):
        for (name, eng), st in [(b, st) for b in builds for st in strides]:
            dm = per_stride[st]
            os.environ["ICRC_AB_PK"] = name[2:] if str(name).startswith("pk") else "0"  # read per launch

            def launch():
                eng.packetize(src.data_ptr(), src.numel(), dm.data_ptr(), nmsg, npk, wire.data_ptr(), npk * st,
                              ln.data_ptr(), ic.data_ptr(), s.cuda_stream)
            launch()
            torch.cuda.synchronize()
            ms = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for _ in range(10):
                    launch()
                b.record(s)
                b.synchronize()
                ms.append(a.elapsed_time(b) / 10)
            med = float(np.median(ms))
            h = (int(ic.sum().item()), int(ln.sum().item()))  # ICRCs and lengths: the same at every stride
            if str(name) in ("-1", "pk0"):
                ref.setdefault("h", h)
            print(json.dumps({"variant": name, "slot_stride": st, "rep": r, "ms_median": round(med, 4),
                              "ms_min": round(min(ms), 4), "GB/s (read+write)": round(alg / (med * 1e-3) / 1e9, 1),
                              "frac_of_8TB/s": round(alg / (med * 1e-3) / 8e12, 4), "same_output": h == ref["h"]}),
                  flush=True)
        ms = []
        for _ in range(5):  # the runtime's own device-to-device copy of the payload bytes, same box
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(10):
                wire[: src.numel()].copy_(src)
            b.record(s)
            b.synchronize()
            ms.append(a.elapsed_time(b) / 10)
        med = float(np.median(ms))
        print(json.dumps({"copy_reference": "d2d copy of the payload bytes", "rep": r, "ms_median": round(med, 4),
                          "GB/s (read+write)": round(2 * src.numel() / (med * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
