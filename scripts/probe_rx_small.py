#!/usr/bin/env python3
"""Latency of one small receive parse (icrc_rx_parse_device): a 16 MiB WRITE's 4096 x 4156-B
packets and 256 x 316-B packets, ragged arrays; median of 5 x 50 calls (HIP events on the stream).

usage: probe_rx_small.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())  # A/B library: diagnostic variants
    s = torch.cuda.current_stream()
    for name, w in (("4096 x 4156 B", workloads.write_message(16 << 20, 4096)),
                    ("256 x 316 B", workloads.write_middle_stream(256, pmtu=256))):
        b = workloads.synthesize(eng, w, stream=s.cuda_stream)
        off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
        desc = torch.zeros(w.n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")

        def call():
            eng.rx_parse(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w.n, desc.data_ptr(), ok.data_ptr(),
                         stream=s.cuda_stream)

        call()
        torch.cuda.synchronize()
        ms = []
        for _ in range(5):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(50):
                call()
            e.record(s)
            e.synchronize()
            ms.append(a.elapsed_time(e) / 50)
        print(json.dumps({"shape": name, "rx_parse_us": round(float(np.median(ms)) * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
