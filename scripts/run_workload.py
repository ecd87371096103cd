#!/usr/bin/env python3
"""Run one workload a few times with the default dispatch (for rocprofv3 --pmc / --stats).

usage: run_workload.py {c1,c1w,c1v,c1vz,c2,c2nr,c2s,c2k,c2m,c3,s316,rx316,rx316r,packetize} [launches] [variant]
  c2nr / c2s / c2k / c2m: C2 without ragged LAST packets / only the 256-B class / only the
  1 KiB class / 256-B and 1 KiB classes (4 Mi packets each, packed, offset / length arrays);
  c1w: C1 compute with write_trailer; c1v / c1vz: C1 verify without / with zero_trailer; s316: 4 Mi strided
  316-byte packets; rx316 / rx316r: icrc_rx_parse_device over those packets (trailers written),
  strided / as a ragged batch; packetize: the fused send packetizer over 192 x 16 MiB WRITE messages
  (786 K x 4156-B packets, as bench.py --extra)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())  # A/B library: diagnostic variants
    if len(sys.argv) > 3:
        eng.set_variant(int(sys.argv[3]))
    s = torch.cuda.current_stream().cuda_stream
    if which in ("rx316", "rx316r"):
        w = workloads.write_middle_stream(1 << 22, pmtu=256)
        L = int(w.lens[0])
        b = workloads.synthesize(eng, w, stream=s)
        o = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        tmp = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, tmp.data_ptr(), True, 0, s)
        desc = torch.empty(w.n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
        if which == "rx316":
            fn = lambda: eng.rx_parse(b.data_ptr(), 0, 0, w.n, desc.data_ptr(), ok.data_ptr(), stride=L, length=L,  # noqa: E731
                                      stream=s)
        else:
            fn = lambda: eng.rx_parse(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, desc.data_ptr(), ok.data_ptr(),  # noqa: E731
                                      stream=s)
    elif which in ("c1", "c1w", "c1v", "c1vz", "s316"):
        w = workloads.write_middle_stream(1 << 22, pmtu=256) if which == "s316" else workloads.write_middle_stream(1 << 20)
        L = int(w.lens[0])
        b = workloads.synthesize(eng, w, stream=s)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        if which in ("c1v", "c1vz"):
            fn = lambda: eng.verify_strided(b.data_ptr(), L, L, w.n, out.data_ptr(), which == "c1vz", s)  # noqa: E731
        else:
            fn = lambda: eng.compute_strided(b.data_ptr(), L, L, w.n, out.data_ptr(), which == "c1w", s)  # noqa: E731
    elif which == "packetize":
        nmsg, mb, pmtu = 192, 16 << 20, 4096
        msgs = icrc_amd.write_messages([dict(local_va=0x7F0000000000 + i * mb, remote_va=0x7E0000000000 + i * mb,
                                             payload_offset=i * mb, total_len=mb, pmtu=pmtu, rkey=3, dqpn=2 + i, psn=0,
                                             msn=i, dst_ip=0xC0A80003, kind=0) for i in range(nmsg)],
                                       slot_stride=56 + pmtu + 4)
        npk = int(msgs["npackets"].sum())
        src = torch.randint(0, 256, (nmsg * mb,), dtype=torch.uint8, device="cuda")
        dm = torch.from_numpy(msgs.view(np.uint8)).cuda()
        wire = torch.empty(npk * (56 + pmtu + 4), dtype=torch.uint8, device="cuda")
        ln = torch.zeros(npk, dtype=torch.int32, device="cuda")
        ic = torch.zeros(npk, dtype=torch.int32, device="cuda")
        fn = lambda: eng.packetize(src.data_ptr(), src.numel(), dm.data_ptr(), nmsg, npk, wire.data_ptr(),  # noqa: E731
                                   wire.numel(), ln.data_ptr(), ic.data_ptr(), s)
    else:
        kw = {"c2": {}, "c2nr": dict(ragged_frac=0.0), "c2s": dict(classes=(256,)), "c2k": dict(classes=(1024,)),
              "c2m": dict(classes=(256, 1024))}
        w = workloads.mixed_mtu_stream(4 << 20, **kw[which]) if which in kw else workloads.write_message(16 << 20, 4096)
        b = workloads.synthesize(eng, w, stream=s)
        o = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        fn = lambda: eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, out.data_ptr(), False, 0, s)  # noqa: E731
    for _ in range(launches):
        fn()
    torch.cuda.synchronize()
    print(f"{which}: {launches} launches done", flush=True)


if __name__ == "__main__":
    main()
