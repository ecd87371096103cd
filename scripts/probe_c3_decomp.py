#!/usr/bin/env python3
"""configs[3] fixed cost, decomposed.  The 16 MiB WRITE (4096 packets, one per
wave of the 256 x 1024-thread grid) through the A/B library's cut kernels, same grid / block / LDS:
  30 / 33 the launch alone without LDS (1024- / 256-thread workgroups), 27 the launch alone,
  28 + the LDS table image, 29 + each wave's (offset, length) load,
  19 the batch kernel's loads only (meta, table, row loads, ring; no CRC), 16 the product kernel.
For compute (with and without write_trailer) and verify (zero_trailer), ragged arrays as bench.py's
configs.c3 passes them, and the same packets as a strided batch of the MIDDLE length.  Prints one
JSON line per (case, variant, round): HIP-event ms per launch over back-to-back launches (the
stream's throughput, launch gaps included).  Run it under rocprofv3 --kernel-trace --stats for
each kernel's own duration."""
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
    Lm = int(np.median(w3.lens))
    cases = {
        "compute_ragged": lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, out.data_ptr(),
                                                    False, 0, s),
        "compute_trailer_ragged": lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n,
                                                            out.data_ptr(), True, 0, s),
        "verify_zero_ragged": lambda: eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w3.n, ok.data_ptr(),
                                                       True, 0, s),
        "compute_strided": lambda: eng.compute_strided(b.data_ptr(), Lm, Lm, w3.n, out.data_ptr(), False, s),
    }
    for rnd in range(2):
        for name, fn in cases.items():
            for v in (30, 33, 27, 28, 29, 19, 16, -1):
                eng.set_variant(v)
                for _ in range(20):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(REPS):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                print(json.dumps({"case": name, "variant": v, "round": rnd,
                                  "us_per_launch": round(e0.elapsed_time(e1) / REPS * 1e3, 2)}), flush=True)
    eng.set_variant(-1)
    eng.close()


if __name__ == "__main__":
    main()
