#!/usr/bin/env python3
"""C3 (16 MiB WRITE round trip, 4096 x 4156-B packets, ragged arrays): per-round-trip time of the
hybrid dispatch (-1), the compacting long walker (224) and the batch kernel alone (16)."""
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
    s = torch.cuda.current_stream().cuda_stream
    w3 = workloads.write_message(16 << 20, 4096)
    b = workloads.synthesize(eng, w3, stream=s)
    off = torch.from_numpy(np.ascontiguousarray(w3.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w3.lens)).cuda()
    out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def rt():
        eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(), True, 0, s)
        eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, ok.data_ptr(), False, 0, s)

    for rnd in range(3):
        for v in (-1, 224, 124, 16):
            eng.set_variant(v)
            for _ in range(10):
                rt()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                rt()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"variant": v, "round": rnd, "ms_per_roundtrip": round(e0.elapsed_time(e1) / 50, 4),
                              "all_ok": bool((ok == 1).all().item())}), flush=True)
    eng.set_variant(-1)


if __name__ == "__main__":
    main()
