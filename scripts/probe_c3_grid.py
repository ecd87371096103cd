#!/usr/bin/env python3
"""configs[3] against the small batch's grid (round 6): the 16 MiB WRITE (4096 x 4156-B packets)
through the A/B library with ICRC_AB_SMALL_PPW = 1 (the product: one packet per wave, 256
workgroups), 2, 4, 8 (fewer workgroups, that many packets per wave on the one-packet pipeline):
whether a launch of fewer waves (its dispatch) beats the burst that more waves put in flight.
Cases as bench.py's configs.c3: compute + write_trailer and verify + zero_trailer (ragged arrays),
and compute alone.  HIP events over REPS back-to-back launches (the stream's rate); results of
every setting compared with PPW 1's.  Run it under rocprofv3 --kernel-trace --stats for each
kernel's own duration (grid sizes tell the settings apart)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402

REPS = int(os.environ.get("C3_REPS", "200"))


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    w3 = workloads.write_message(16 << 20, 4096)
    b = workloads.synthesize(eng, w3, stream=s)
    off = torch.from_numpy(np.ascontiguousarray(w3.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w3.lens)).cuda()
    out = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
    ok = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")

    def compute():
        eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(), False, 0, s)

    def roundtrip():
        eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(), True, 0, s)
        eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, ok.data_ptr(), True, 0, s)

    def gpu_rate(fn, k=16, reps=5):  # bench.py's configs.c3 method: launches queued behind a spin kernel
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
    for rnd in range(int(os.environ.get("C3_ROUNDS", "2"))):
        for ppw in (1, 2, 4, 8) if rnd < 1 else (1, 2):
            os.environ["ICRC_AB_SMALL_PPW"] = str(ppw)
            row = {"round": rnd, "packets_per_wave": ppw}
            for name, fn in (("compute", compute), ("roundtrip", roundtrip)):
                for _ in range(20):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(REPS):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                row[name + "_us"] = round(e0.elapsed_time(e1) / REPS * 1e3, 2)
            row["gpu_us_compute_trailer"] = gpu_rate(
                lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(), True, 0, s))
            row["gpu_us_verify_zero"] = gpu_rate(
                lambda: eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, ok.data_ptr(), True, 0, s))
            roundtrip()  # (the verify-rate launches above zeroed the trailers: write them again, check them once)
            torch.cuda.synchronize()
            got = (out.cpu().numpy().tobytes(), ok.cpu().numpy().tobytes(), b[:4096 * 8].cpu().numpy().tobytes())
            ref = ref or got
            row["same_results"] = got == ref
            row["all_ok"] = bool((ok == 1).all().item())
            print(json.dumps(row), flush=True)
    os.environ.pop("ICRC_AB_SMALL_PPW", None)
    eng.close()


if __name__ == "__main__":
    main()
