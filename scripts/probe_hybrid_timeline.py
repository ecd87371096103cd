"""probe_hybrid_timeline.py — when the fused hybrid kernel's long-packet workgroups run against the
oct workgroups' ends (VERDICT r03 Next #2: "the oct workgroups' end-time distribution vs the long
workgroups' start").  A/B library, ICRC_AB_HYBRID_STAMP=1: every workgroup stores its start / end
(s_memrealtime, 100 MHz) and kind in a device array, read back with icrc_ab_hybrid_stamps.

usage: JOBS=C2,C2nr REPS=5 python3 scripts/probe_hybrid_timeline.py
(WALKS=...: the ICRC_AB_LONG_WALK forms of the long-packet walk measured in round 4, since removed:
0 the product's; 1 three packets in flight; 2 the next (offset, length) block prefetched; 3 both,
profiles/r04_hybrid_timeline_walks.jsonl.)  Prints one JSON line per (job, repetition): the mean
of 10 launches (events) and the last launch's workgroup times in us from its first workgroup's start."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def pct(a, q):
    return round(float(np.percentile(a, q)), 1) if len(a) else None


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    kws = {"C2": {}, "C2nr": dict(ragged_frac=0.0)}
    for name in os.environ.get("JOBS", "C2,C2nr").split(","):
        w = workloads.mixed_mtu_stream(4 << 20, **kws[name])
        b = workloads.synthesize(eng, w, stream=s)
        o, ln = dev(w.off), dev(w.lens)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")

        def run():
            eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, out.data_ptr(), False, 0, s)

        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        os.environ["ICRC_AB_HYBRID_STAMP"] = "1"
        for rep in range(int(os.environ.get("REPS", "5"))):
            for walk in os.environ.get("WALKS", "0").split(","):
                os.environ["ICRC_AB_LONG_WALK"] = walk
                for _ in range(2):
                    run()
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                tail = np.zeros(5 * 8192, dtype=np.uint32)
                rc = eng._lib.icrc_ab_hybrid_stamps(tail.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 8192)
                tail = tail.reshape(8192, 5)
                grid = int(np.count_nonzero(tail[:, 1]))  # the launch's workgroups (the array starts zeroed)
                tail = tail[:grid]
                if rc != 0 or grid == 0 or not (tail[0, 4] == 0 and tail[-1, 4] == 1):
                    print(json.dumps({"job": name, "rep": rep, "walk": walk, "error": "no stamps", "rc": rc}), flush=True)
                    continue
                t0 = (tail[:, 0].astype(np.uint64) | (tail[:, 1].astype(np.uint64) << np.uint64(32))).astype(np.float64)
                t1 = (tail[:, 2].astype(np.uint64) | (tail[:, 3].astype(np.uint64) << np.uint64(32))).astype(np.float64)
                base = t0.min()
                st, en = (t0 - base) * TICK_US, (t1 - base) * TICK_US
                octm, lngm = tail[:, 4] == 0, tail[:, 4] == 1
                span = float(en.max())
                busy_long = en[lngm] - st[lngm]
                ncu = int(octm.sum())
                print(json.dumps({
                    "job": name, "rep": rep, "walk": walk, "packets": int(w.n), "grid_oct": ncu,
                    "grid_long": int(lngm.sum()), "ms_events_10": round(ms, 4),
                    "span_us_stamps_last": round(span, 1),
                    "oct_end_us": {"min": pct(en[octm], 0), "p10": pct(en[octm], 10), "p50": pct(en[octm], 50),
                                   "p90": pct(en[octm], 90), "max": pct(en[octm], 100)},
                    "long_start_us": {"min": pct(st[lngm], 0), "p50": pct(st[lngm], 50), "max": pct(st[lngm], 100)},
                    "long_end_us": {"min": pct(en[lngm], 0), "p50": pct(en[lngm], 50), "max": pct(en[lngm], 100)},
                    "long_busy_us": {"min": pct(busy_long, 0), "p50": pct(busy_long, 50), "max": pct(busy_long, 100)},
                    "after_last_oct_us": round(span - float(en[octm].max()), 1),
                    "cu_idle_frac": round(1.0 - float((en - st).sum()) / (ncu * span), 4),
                }), flush=True)
        del b, o, ln, out
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
