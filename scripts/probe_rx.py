#!/usr/bin/env python3
"""The receive parse (verify pass + icrc_rx_desc_kernel) on 786 K ragged 4156-byte WRITE_MIDDLE
packets and on 4 Mi ragged 316-byte ones: one JSON line per shape with the event-timed rx_parse
call; run under `rocprofv3 --kernel-trace --stats` for the two passes separately.

usage: probe_rx.py [reps] [engine variant ...]   (default: -1 = the default dispatch; 301 / 302
the fused single pass on every batch, a store per packet / descriptors per 64-packet block)"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    variants = [int(v) for v in sys.argv[2:]] or [-1]
    # the product library (ICRC_AMD_LIB selects another build for a two-build A/B)
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    for name, w in (("786K x 4156 B", workloads.write_middle_stream(786432)),
                    ("4Mi x 316 B", workloads.write_middle_stream(1 << 22, pmtu=256))):
        b = workloads.synthesize(eng, w, stream=s)
        off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
        for _, v in [(r, v) for r in range(2) for v in variants]:
            eng.set_variant(v)
            d = torch.full((w.n * icrc_amd.RX_DESC_DTYPE.itemsize,), 0xEE, dtype=torch.uint8, device="cuda")
            fn = lambda: eng.rx_parse(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w.n, d.data_ptr(),  # noqa: E731
                                      ok.data_ptr(), stream=s)
            fn()
            torch.cuda.synchronize()
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(e) / reps
            desc = d.cpu().numpy().view(icrc_amd.RX_DESC_DTYPE)
            print(json.dumps({"shape": name, "variant": v, "rx_parse_ms": round(ms, 4), "all_ok": bool(np.all(desc["icrc_ok"] == 1)),
                              "status_ok": bool(np.all(desc["status"] == 0))}), flush=True)
        del b


if __name__ == "__main__":
    main()
