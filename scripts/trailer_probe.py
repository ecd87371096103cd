#!/usr/bin/env python3
"""C1 (1 Mi x 4156 B, strided and ragged): compute with / without the trailer write and verify
with / without in-place trailer zeroing — the cost of a per-packet store inside the CRC pipeline."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
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
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())  # A/B library: diagnostic variants
    s = torch.cuda.current_stream().cuda_stream
    n = 1 << 20
    w = workloads.write_middle_stream(n)
    L = int(w.lens[0])
    b = workloads.synthesize(eng, w, stream=s)
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
    cases = {
        "compute": lambda: eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(), False, s),
        "compute_trailer": lambda: eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(), True, s),
        "verify": lambda: eng.verify_strided(b.data_ptr(), L, L, n, ok.data_ptr(), False, s),
        "compute_ragged_trailer": lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n,
                                                            out.data_ptr(), True, 0, s),
        "verify_zero": lambda: (eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(), True, s),
                                eng.verify_strided(b.data_ptr(), L, L, n, ok.data_ptr(), True, s)),
    }
    for rnd in range(2):
        for name, fn in cases.items():
            ms = timed(fn)
            print(json.dumps({"case": name, "round": rnd, "ms": round(ms, 4),
                              "GB/s": round(n * L / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
