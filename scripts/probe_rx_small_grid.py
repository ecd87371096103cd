#!/usr/bin/env python3
"""The small-batch receive (icrc_rx_kernel, one fused pass: verify + descriptors) against its grid
(round 6): configs[3]'s 16 MiB WRITE (4096 x 4156-B packets, trailers written) received through
icrc_rx_parse_device with ICRC_AB_RX_SMALL_PPW = 1 (the product: one packet per wave), 2, 4 — the
change the compute dispatch took for its small batches (probe_c3_grid.py).  The A/B library; HIP
events over launches queued behind a spin kernel (bench.py's configs.c3 method), five rounds
alternating; descriptors and ok bytes of every setting compared with PPW 1's."""
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
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    w3 = workloads.write_message(16 << 20, 4096)
    b = workloads.synthesize(eng, w3, stream=s)
    off = torch.from_numpy(np.ascontiguousarray(w3.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w3.lens)).cuda()
    out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(), True, 0, s)
    desc = torch.zeros(w3.n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def rx():
        eng.rx_parse(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, desc.data_ptr(), ok.data_ptr(), stream=s)

    def gpu_rate(fn, k=16, reps=5):
        res = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(4_000_000)
            e0.record()
            for _ in range(k):
                fn()
            e1.record()
            e1.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / k)
        return round(float(np.median(res)), 2)

    ref = None
    for rnd in range(5):
        for ppw in (1, 2, 4) if rnd == 0 else (1, 2):
            os.environ["ICRC_AB_RX_SMALL_PPW"] = str(ppw)
            for _ in range(20):
                rx()
            torch.cuda.synchronize()
            row = {"round": rnd, "packets_per_wave": ppw, "gpu_us_rx_parse": gpu_rate(rx)}
            desc.zero_()
            ok.zero_()
            rx()
            torch.cuda.synchronize()
            got = (desc.cpu().numpy().tobytes(), ok.cpu().numpy().tobytes())
            ref = ref or got
            row["same_results"] = got == ref
            row["all_ok"] = bool((ok == 1).all().item())
            print(json.dumps(row), flush=True)
    os.environ.pop("ICRC_AB_RX_SMALL_PPW", None)
    eng.close()


if __name__ == "__main__":
    main()
