"""probe_presort.py — what would a larger sort window buy the short-packet kernel on C2?  The oct
kernel sorts each 64-packet block by row count, and the sets of eight at class boundaries are mixed
(25 % of C2's sets: 16 % more row steps issued than useful, tests-side simulation).  Here the
(offset, length) arrays themselves are pre-sorted by row count within windows of W packets
(W = 64: what the kernel does anyway; 128, 256, 1024; 'all': one global order), so the kernel's
64-packet blocks see the order a W-packet sort would give.  Same packets, same buffer; only the
order of the arrays changes (the ICRCs come out permuted and are checked against the original
order's).  Prints one JSON line per window: median / min of ROUNDS x 10 launches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    w = workloads.mixed_mtu_stream(4 << 20)
    b = workloads.synthesize(eng, w, stream=s)
    L = w.lens.astype(np.int64)
    R = np.where(L <= 1088, (1 + (L - 4) // 4 + 7) // 8, 63)
    nb = int(L.sum())
    orders = {"orig": np.arange(w.n)}
    for W in (64, 128, 256, 1024):
        idx = np.arange(w.n)
        key = (idx // W) * 128 + R  # stable sort by (window, R)
        orders[str(W)] = np.argsort(key, kind="stable")
    orders["all"] = np.argsort(R, kind="stable")
    runs = {}
    for name, perm in orders.items():
        o = torch.from_numpy(np.ascontiguousarray(w.off[perm])).cuda()
        l = torch.from_numpy(np.ascontiguousarray(w.lens[perm])).cuda()
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        runs[name] = (perm, o, l, out)
    times = {k: [] for k in runs}
    ref = None
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for name, (perm, o, l, out) in runs.items():
            fn = lambda: eng.compute_batch(b.data_ptr(), o.data_ptr(), l.data_ptr(), w.n, out.data_ptr(), False, 0, s)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 10)
            got = np.empty(w.n, np.uint32)
            got[perm] = out.cpu().numpy().view(np.uint32)
            if ref is None:
                ref = got.copy()
            assert np.array_equal(got, ref), name
    for name, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"window": name, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "frac_of_8TB": round(nb / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
