#!/usr/bin/env python3
"""The sparse long-packet walk, A/B on one box (round 6): ICRC_AB_LONG_WALK=1 (run_walk_masked: the
wave's lengths scanned 1024 at a time, each long packet's meta one packet ahead) against 0 (the
product's walker, run_pipelined_long: a drained meta round trip per 64-packet block), through the
A/B library, on
configs[2]'s batch (mixed_mtu_stream(4 Mi)): compute (the hybrid launch) and the receive parse
(the ragged one-pass receive).  The env knob is read per call, so both run alternately in one
process.  Median of 5 x 10 launches, HIP events on the launch stream; results compared between
the two walkers (ICRCs, ok bytes, descriptors)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def timed(fn, s):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(10):
            fn()
        b.record(s)
        b.synchronize()
        ms.append(a.elapsed_time(b) / 10)
    return float(np.median(ms))


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream()
    wm = workloads.mixed_mtu_stream(4 << 20)
    d_buf = workloads.synthesize(eng, wm, stream=s.cuda_stream)
    d_off = torch.from_numpy(np.ascontiguousarray(wm.off)).cuda()
    d_len = torch.from_numpy(np.ascontiguousarray(wm.lens)).cuda()
    d_out = torch.zeros(wm.n, dtype=torch.int32, device="cuda")
    eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n, d_out.data_ptr(), True, 0,
                      s.cuda_stream)  # trailers written: the receive legs verify them
    torch.cuda.synchronize()
    d_desc = torch.zeros(wm.n * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(wm.n, dtype=torch.uint8, device="cuda")
    tot = int(wm.lens.astype(np.uint64).sum())
    ref = {}
    for rnd in range(3):
        for walk in ("1", "0"):
            os.environ["ICRC_AB_LONG_WALK"] = walk
            c = timed(lambda: eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n,
                                                d_out.data_ptr(), False, 0, s.cuda_stream), s)
            r = timed(lambda: eng.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), wm.n, d_desc.data_ptr(),
                                           d_ok.data_ptr(), stream=s.cuda_stream), s)
            h = (d_out.cpu().numpy().tobytes(), d_ok.cpu().numpy().tobytes(), d_desc.cpu().numpy().tobytes())
            ref.setdefault("h", h)
            print(json.dumps({"round": rnd, "long_walk": walk, "c2_compute_ms": round(c, 4),
                              "c2_compute_frac": round(tot / (c * 1e-3) / 8e12, 4), "c2_rx_ms": round(r, 4),
                              "c2_rx_frac": round((tot + 73 * wm.n) / (r * 1e-3) / 8e12, 4),
                              "same_results": h == ref["h"], "all_ok": bool((d_ok == 1).all().item())}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
