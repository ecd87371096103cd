"""probe_split.py — the hybrid dispatch's length split on C2 (A/B library, ICRC_AB_SPLIT read per
launch): the oct kernel takes L < split, the long-packet kernel L >= split.  The default split is
1089 (every packet the oct kernel can hold); lower splits move the 1 KiB class (1084 B) and the
longer ragged packets to the long-packet kernel.  One process, interleaved rounds; prints one JSON
line per (workload, split) with the median of ROUNDS x 10 launches, results checked equal."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    splits = [int(x) for x in os.environ.get("SPLITS", "1089,1000,700,400,320").split(",")]
    jobs = {}
    for name, kw in (("C2", {}), ("C2m", dict(classes=(256, 1024)))):
        w = workloads.mixed_mtu_stream(4 << 20, **kw)
        b = workloads.synthesize(eng, w, stream=s)
        o, l = dev(w.off), dev(w.lens)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        jobs[name] = (b, o, l, out, w.n, int(w.lens.astype(np.uint64).sum()))
    times = {(j, sp): [] for j in jobs for sp in splits}
    ref = {}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for sp in splits:
            os.environ["ICRC_AB_SPLIT"] = str(sp)
            for j, (b, o, l, out, n, nb) in jobs.items():
                fn = lambda: eng.compute_batch(b.data_ptr(), o.data_ptr(), l.data_ptr(), n, out.data_ptr(), False, 0, s)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, sp)].append(e0.elapsed_time(e1) / 10)
                got = out.cpu().numpy().copy()
                ref.setdefault(j, got)
                assert np.array_equal(ref[j], got), (j, sp)
    for (j, sp), ts in times.items():
        nb = jobs[j][5]
        med = float(np.median(ts))
        print(json.dumps({"workload": j, "split": sp, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "frac_of_8TB": round(nb / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
