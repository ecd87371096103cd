#!/usr/bin/env python3
"""A/B the ICRC kernel variants in ONE process, interleaved rounds (methodology rule 24):
C1 (1 Mi x 4156 B, strided) and C2 (mixed MTU, ragged) for each variant; checks that every
variant returns identical ICRCs.  Prints one JSON line per (workload, variant)."""
DIAGNOSTIC = {15, 18, 19, 21, 22, 23, 41, 42, 43, 44, 45, 46, 47, 48, 50, 53}  # ablations (loads-only / CRC-only / no loads): wrong results by design
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402

GIB = float(1 << 30)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def main():
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "16,13,0").split(",")]
    rounds = int(os.environ.get("ROUNDS", "5"))
    launches = int(os.environ.get("LAUNCHES", "10"))
    # the product library (or ICRC_AMD_LIB's build) unless a variant exists only in the A/B build
    ab_only = any(v % 100 in DIAGNOSTIC or v % 100 in (49, 51, 52) for v in variants if v >= 0)
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library() if ab_only else None)
    s = torch.cuda.current_stream().cuda_stream
    jobs = {}
    keep = []
    for name in os.environ.get("JOBS", "C1,C2").split(","):
        if name in ("C1v", "S316v"):  # verify (is_icrc_valid) of the strided batches, trailers written first
            w1 = workloads.write_middle_stream(1 << 22, pmtu=256) if name == "S316v" else workloads.write_middle_stream(1 << 20)
            L = int(w1.lens[0])
            b1 = workloads.synthesize(eng, w1, stream=s)
            scratch = torch.zeros(w1.n, dtype=torch.int32, device="cuda")
            eng.compute_strided(b1.data_ptr(), L, L, w1.n, scratch.data_ptr(), True, s)  # write the trailers
            ok1 = torch.zeros(w1.n, dtype=torch.uint8, device="cuda")
            keep += [b1, scratch, ok1]
            jobs[name] = (lambda b1=b1, ok1=ok1, n=w1.n, L=L: eng.verify_strided(b1.data_ptr(), L, L, n, ok1.data_ptr(),
                                                                               False, s), w1.n * L, ok1)
            continue
        if name in ("C1", "S316"):  # S316: 4 Mi strided 316-byte packets (the 256-B MTU class)
            w1 = workloads.write_middle_stream(1 << 22, pmtu=256) if name == "S316" else workloads.write_middle_stream(1 << 20)
            L = int(w1.lens[0])
            b1 = workloads.synthesize(eng, w1, stream=s)
            out1 = torch.zeros(w1.n, dtype=torch.int32, device="cuda")
            keep += [b1, out1]
            jobs[name] = (lambda b1=b1, out1=out1, n=w1.n, L=L: eng.compute_strided(b1.data_ptr(), L, L, n, out1.data_ptr(),
                                                                                   False, s), w1.n * L, out1)
            continue
        if name in ("C3", "C3c") or name.startswith("W"):
            # 16 MiB WRITE: compute (write trailers) + verify (zero trailers) / compute only;
            # Wk: a WRITE of k 4 KiB packets, compute only (as C3c)
            w3 = workloads.write_message((int(name[1:]) if name.startswith("W") else 4096) * 4096, 4096)
            b3 = workloads.synthesize(eng, w3, stream=s)
            o3, l3 = dev(w3.off), dev(w3.lens)
            out3 = torch.zeros(w3.n, dtype=torch.int32, device="cuda")
            ok3 = torch.zeros(w3.n, dtype=torch.uint8, device="cuda")
            keep += [b3, o3, l3, out3, ok3]

            def rt(b3=b3, o3=o3, l3=l3, out3=out3, ok3=ok3, n=w3.n, both=name == "C3"):
                eng.compute_batch(b3.data_ptr(), o3.data_ptr(), l3.data_ptr(), n, out3.data_ptr(), both, 0, s)
                if both:
                    eng.verify_batch(b3.data_ptr(), o3.data_ptr(), l3.data_ptr(), n, ok3.data_ptr(), True, 0, s)
            nb3 = int(w3.lens.astype(np.uint64).sum()) * (2 if name == "C3" else 1)
            if name.startswith("W"):
                name = f"W{w3.n}"
            jobs[name] = (rt, nb3, out3)
            continue
        if name in ("C2short", "C2long"):  # the C2 batch's own packets of one half only (same buffer, same
            # offsets): L <= 1088 (the oct half) / L >= 1089 (the long-packet half) — the mix decomposition
            w2 = workloads.mixed_mtu_stream(4 << 20)
            b2 = workloads.synthesize(eng, w2, stream=s)
            sel = (w2.lens <= 1088) if name == "C2short" else (w2.lens >= 1089)
            off_s, len_s = np.ascontiguousarray(w2.off[sel]), np.ascontiguousarray(w2.lens[sel])
            o2, l2 = dev(off_s), dev(len_s)
            out2 = torch.zeros(int(sel.sum()), dtype=torch.int32, device="cuda")
            keep += [b2, o2, l2, out2]
            jobs[name] = (lambda b2=b2, o2=o2, l2=l2, out2=out2, n=int(sel.sum()): eng.compute_batch(
                b2.data_ptr(), o2.data_ptr(), l2.data_ptr(), n, out2.data_ptr(), False, 0, s),
                int(len_s.astype(np.uint64).sum()), out2)
            continue
        if name == "R4K":  # C1's packets as a ragged batch (offset / length arrays)
            w2 = workloads.write_middle_stream(1 << 20)
            b2 = workloads.synthesize(eng, w2, stream=s)
            o2, l2 = dev(w2.off), dev(w2.lens)
            out2 = torch.zeros(w2.n, dtype=torch.int32, device="cuda")
            keep += [b2, o2, l2, out2]
            jobs[name] = (lambda b2=b2, o2=o2, l2=l2, out2=out2, n=w2.n: eng.compute_batch(
                b2.data_ptr(), o2.data_ptr(), l2.data_ptr(), n, out2.data_ptr(), False, 0, s),
                int(w2.lens.astype(np.uint64).sum()), out2)
            continue
        kw = {"C2": {}, "C2k": dict(classes=(1024,)), "C2s": dict(classes=(256,)), "C2nr": dict(ragged_frac=0.0),
              "C2m": dict(classes=(256, 1024)), "C2snr": dict(classes=(256,), ragged_frac=0.0)}[name]
        w2 = workloads.mixed_mtu_stream(4 << 20, **kw)
        b2 = workloads.synthesize(eng, w2, stream=s)
        o2, l2 = dev(w2.off), dev(w2.lens)
        out2 = torch.zeros(w2.n, dtype=torch.int32, device="cuda")
        keep += [b2, o2, l2, out2]
        jobs[name] = (lambda b2=b2, o2=o2, l2=l2, out2=out2, n=w2.n: eng.compute_batch(
            b2.data_ptr(), o2.data_ptr(), l2.data_ptr(), n, out2.data_ptr(), False, 0, s),
            int(w2.lens.astype(np.uint64).sum()), out2)
    times = {(j, v): [] for j in jobs for v in variants}
    ref = {}
    for r in range(rounds):
        for v in variants:
            eng.set_variant(v)
            for j, (fn, nb, out) in jobs.items():
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(launches):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, v)].append(e0.elapsed_time(e1) / launches)
                if v % 100 in DIAGNOSTIC:
                    continue  # diagnostic ablations (loads-only / CRC-only) are wrong by design
                got = out.cpu().numpy().copy()
                if j not in ref:
                    ref[j] = got
                assert np.array_equal(ref[j], got), f"variant {v} differs on {j}"
    for (j, v), ts in times.items():
        nb = jobs[j][1]
        med = float(np.median(ts))
        print(json.dumps({"workload": j, "variant": v, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "GB/s": round(nb / (med * 1e-3) / 1e9, 1), "frac_of_8TB": round(nb / (med * 1e-3) / 8e12, 4)}))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
