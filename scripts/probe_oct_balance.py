#!/usr/bin/env python3
"""Load balance of the oct kernel's persistent waves: diagnostic variant 53 (A/B library) runs the
full oct kernel and has every wave stamp its start and end (s_memrealtime, 100 MHz) over its first
four results.  For each workload: the kernel time of variant 40 (the oct kernel, forced), the span
of the stamps, and the spread of the waves' end times (per wave, per workgroup = CU).  If every
wave ended at the mean end time the kernel would take about mean_end instead of the span.
Prints one JSON line per workload."""
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
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for name in os.environ.get("JOBS", "C2m,C2s,S316").split(","):
        if name == "S316":
            w = workloads.write_middle_stream(1 << 22, pmtu=256)
        else:
            w = workloads.mixed_mtu_stream(4 << 20, classes={"C2m": (256, 1024), "C2s": (256,), "C2k": (1024,)}[name])
        b = workloads.synthesize(eng, w, stream=s)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        if name == "S316":
            L = int(w.lens[0])
            fn = lambda: eng.compute_strided(b.data_ptr(), L, L, w.n, out.data_ptr(), False, s)  # noqa: E731
        else:
            o, ln = torch.from_numpy(w.off).cuda(), torch.from_numpy(w.lens).cuda()
            fn = lambda: eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, out.data_ptr(), False, 0, s)  # noqa: E731
        res = {"workload": name, "n": int(w.n)}
        for v in (40, 53):
            eng.set_variant(v)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[f"ms_v{v}"] = round(e0.elapsed_time(e1) / 10, 4)
        eng.set_variant(53)
        runs = []
        for _ in range(2):
            fn()
            torch.cuda.synchronize()
            runs.append(out.cpu().numpy().view(np.uint32).copy())
        r = runs[0]
        grid = min((w.n + 15) // 16, ncu)
        tw = grid * 16
        chunk = (w.n + tw - 1) // tw
        chunk = (chunk + 63) & ~63 if chunk > 32 else (chunk + 7) & ~7
        # the waves' ranges as wave_range (icrc_device.h) forms them, with the oct skew in force
        e = int(os.environ.get("ICRC_AB_SKEW_OCT", str(45 | 3 << 12)))
        unit, e = 8 << ((e >> 12) & 3), e & 0xFFF
        U = 16 * chunk // unit

        def start(k):
            f, r = k >> 2, k & 3
            return U * (1024 * k + e * (4 * f * (4 - f) + r * (3 - 2 * f))) // (16 * 1024)
        los = np.array([g * 16 * chunk + unit * start(k) for g in range(grid) for k in range(16)], dtype=np.int64) \
            if e and chunk >= 64 else np.arange(0, w.n, chunk)
        los = los[los < w.n]
        t0 = r[los].astype(np.uint64) | (r[los + 1].astype(np.uint64) << np.uint64(32))
        t1 = r[los + 2].astype(np.uint64) | (r[los + 3].astype(np.uint64) << np.uint64(32))
        base = t0.min()
        s0, s1 = (t0 - base).astype(np.float64) / 100.0, (t1 - base).astype(np.float64) / 100.0  # us
        wg = los // (16 * chunk)
        wg_end = np.array([s1[wg == g].max() for g in np.unique(wg)])
        res.update({"waves": int(los.size), "chunk": int(chunk), "span_us": round(float(s1.max()), 2),
                    "start_us_max": round(float(s0.max()), 2),
                    "wave_end_us": {q: round(float(np.percentile(s1, q)), 2) for q in (0, 10, 50, 90, 99, 100)},
                    "wave_end_mean_us": round(float(s1.mean()), 2),
                    "cu_end_us": {q: round(float(np.percentile(wg_end, q)), 2) for q in (0, 10, 50, 90, 100)},
                    "cu_end_mean_us": round(float(wg_end.mean()), 2)})
        # is the unevenness tied to the wave's slot (deterministic) or random run to run?
        slot = np.arange(los.size) % 16
        res["end_by_wave_slot_us"] = [round(float(s1[slot == k].mean()), 1) for k in range(16)]
        xcd = wg % 8
        res["end_by_xcd_us"] = [round(float(s1[xcd == k].mean()), 1) for k in range(8)]
        r2 = runs[1]
        u0 = r2[los].astype(np.uint64) | (r2[los + 1].astype(np.uint64) << np.uint64(32))
        u1 = r2[los + 2].astype(np.uint64) | (r2[los + 3].astype(np.uint64) << np.uint64(32))
        d1, d2 = (t1 - t0).astype(np.float64), (u1 - u0).astype(np.float64)
        res["wave_duration_corr_between_runs"] = round(float(np.corrcoef(d1, d2)[0, 1]), 3)
        print(json.dumps(res))
        sys.stdout.flush()
        del b, out


if __name__ == "__main__":
    main()
