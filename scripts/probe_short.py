#!/usr/bin/env python3
"""Time the short-packet kernels on uniform batches (one length), strided and ragged, beside C2:
separates per-packet cost from C2's length mix.  usage: probe_short.py VARIANTS (comma list)."""
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
    variants = [int(v) for v in sys.argv[1].split(",")]
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())  # A/B library: diagnostic variants
    s = torch.cuda.current_stream().cuda_stream
    jobs = {}
    for pmtu in (256, 1024):
        w = workloads.write_middle_stream(1 << 22 if pmtu == 256 else 1 << 20, pmtu=pmtu)
        L = int(w.lens[0])
        b = workloads.synthesize(eng, w, stream=s)
        o, ln = torch.from_numpy(w.off.copy()).cuda(), torch.from_numpy(w.lens.copy()).cuda()
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        jobs[f"strided{L}"] = (lambda b=b, L=L, w=w, out=out: eng.compute_strided(
            b.data_ptr(), L, L, w.n, out.data_ptr(), False, s), w.n * L)
        jobs[f"ragged{L}"] = (lambda b=b, o=o, ln=ln, w=w, out=out: eng.compute_batch(
            b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, out.data_ptr(), False, 0, s), w.n * L)
    w = workloads.mixed_mtu_stream(4 << 20)
    b2 = workloads.synthesize(eng, w, stream=s)
    o2, ln2 = torch.from_numpy(np.ascontiguousarray(w.off)).cuda(), torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
    out2 = torch.zeros(w.n, dtype=torch.int32, device="cuda")
    jobs["c2"] = (lambda: eng.compute_batch(b2.data_ptr(), o2.data_ptr(), ln2.data_ptr(), w.n, out2.data_ptr(), False, 0, s),
                  int(w.lens.astype(np.int64).sum()))
    times = {(j, v): [] for j in jobs for v in variants}
    for _ in range(5):
        for v in variants:
            eng.set_variant(v)
            for j, (fn, nb) in jobs.items():
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, v)].append(e0.elapsed_time(e1) / 10)
    for (j, v), ts in times.items():
        med = float(np.median(ts))
        nb = jobs[j][1]
        print(json.dumps({"job": j, "variant": v, "ms": round(med, 4), "TB/s": round(nb / med / 1e9, 3)}))
    eng.set_variant(-1)


if __name__ == "__main__":
    main()
