#!/usr/bin/env python3
"""Receive-parse and verify rates on the C1 batch: ragged (off/len arrays) vs strided, and the
plain verify kernel, to locate the receive path's losses.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    n = 1 << 20
    w = workloads.write_middle_stream(n)
    L = int(w.lens[0])
    b = workloads.synthesize(eng, w, stream=s)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_strided(b.data_ptr(), L, L, n, d_out.data_ptr(), True, s)
    off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
    desc = torch.empty(n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cases = {
        "rx_ragged": lambda: eng.rx_parse(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, desc.data_ptr(), ok.data_ptr(), stream=s),
        "rx_strided": lambda: eng.rx_parse(b.data_ptr(), 0, 0, n, desc.data_ptr(), ok.data_ptr(), stride=L, length=L, stream=s),
        "verify_strided": lambda: eng.verify_strided(b.data_ptr(), L, L, n, ok.data_ptr(), False, s),
        "verify_ragged": lambda: eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, ok.data_ptr(), False, 0, s),
        "compute_ragged": lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, d_out.data_ptr(), False, 0, s),
    }
    for name, fn in cases.items():
        ms = timed(fn)
        print(json.dumps({"case": name, "ms": round(ms, 4), "GB/s": round(n * L / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
