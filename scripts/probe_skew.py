#!/usr/bin/env python3
"""Sweep of the persistent waves' work skew (BatchParams::skew, ICRC_AB_SKEW in the A/B library,
read per call) in ONE process, interleaved rounds: C1 (strided 4156 B), C2 (mixed MTU, hybrid
launch), S316 (strided 316 B, oct), C2k (1 KiB class).  Every skew must return the same results.
Prints one JSON line per (workload, skew)."""
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
    # an entry "e" skews both kernels by e, "a/b" the oct kernel by a and the one-packet pipeline by b
    skews = (sys.argv[1] if len(sys.argv) > 1 else "0,30,45,60,90").split(",")
    rounds = int(os.environ.get("ROUNDS", "3"))
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    jobs, keep = {}, []
    for name in os.environ.get("JOBS", "C1,C2,S316,C2k").split(","):
        if name == "C1v":  # verify (is_icrc_valid) of C1, trailers written first
            w = workloads.write_middle_stream(1 << 20)
            L = int(w.lens[0])
            b = workloads.synthesize(eng, w, stream=s)
            scratch = torch.zeros(w.n, dtype=torch.int32, device="cuda")
            eng.compute_strided(b.data_ptr(), L, L, w.n, scratch.data_ptr(), True, s)
            ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
            keep += [b, scratch, ok]
            jobs[name] = (lambda b=b, ok=ok, n=w.n, L=L: eng.verify_strided(b.data_ptr(), L, L, n, ok.data_ptr(), False, s),
                          w.n * L, ok)
            continue
        if name in ("C1", "S316"):
            w = workloads.write_middle_stream(1 << 22, pmtu=256) if name == "S316" else workloads.write_middle_stream(1 << 20)
            L = int(w.lens[0])
            b = workloads.synthesize(eng, w, stream=s)
            out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
            keep += [b, out]
            jobs[name] = (lambda b=b, out=out, n=w.n, L=L: eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(), False, s),
                          w.n * L, out)
            continue
        w = workloads.mixed_mtu_stream(4 << 20, **({"C2k": dict(classes=(1024,))}.get(name, {})))
        b = workloads.synthesize(eng, w, stream=s)
        o, ln = torch.from_numpy(w.off).cuda(), torch.from_numpy(w.lens).cuda()
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        keep += [b, o, ln, out]
        jobs[name] = (lambda b=b, o=o, ln=ln, out=out, n=w.n: eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), n,
                                                                                out.data_ptr(), False, 0, s),
                      int(w.lens.astype(np.uint64).sum()), out)
    times = {(j, k): [] for j in jobs for k in skews}
    ref = {}
    for _ in range(rounds):
        for k in skews:
            a, _, b = k.partition("/")
            os.environ["ICRC_AB_SKEW_OCT"], os.environ["ICRC_AB_SKEW_LONG"] = a, b or a
            for j, (fn, nb, out) in jobs.items():
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, k)].append(e0.elapsed_time(e1) / 10)
                got = out.cpu().numpy().copy()
                if j not in ref:
                    ref[j] = got
                assert np.array_equal(ref[j], got), f"skew {k} differs on {j}"
    for (j, k), ts in times.items():
        print(json.dumps({"workload": j, "skew": k, "ms_median": round(float(np.median(ts)), 4), "ms_min": round(min(ts), 4),
                          "ms_all": [round(t, 4) for t in ts]}))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
