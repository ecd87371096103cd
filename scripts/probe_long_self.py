#!/usr/bin/env python3
"""A/B: the hybrid launch's long packets walked by a second set of long-packet workgroups
(ICRC_AB_LONG_SELF=0, the round-4 form) or by each workgroup itself after its oct range (the
default since round 5: the W = 64 image reloaded into LDS, no second set, no tail); FORMS picks
the forms ("0", "1", "s2" = in place with 2 x #CUs workgroups, "k45" = in place with oct wave
skew 45, ...).  One process,
alternating rounds; configs[2], C1's packets as a ragged batch, the 316-B class alone; the results
of both forms must be identical.  One JSON line per (batch, form): median ms of ROUNDS x 10 launches."""
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
    rounds = int(os.environ.get("ROUNDS", "5"))
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    batches = {
        "C2": workloads.mixed_mtu_stream(4 << 20),
        "R4K": workloads.write_middle_stream(1 << 20),
        "R316": workloads.write_middle_stream(4 << 20, pmtu=256),
    }
    for name, w in batches.items():
        b = workloads.synthesize(eng, w, stream=s)
        off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        forms = os.environ.get("FORMS", "0,1").split(",")  # LONG_SELF value, or "s<k>": in place, k x #CUs workgroups
        out = {f: torch.zeros(w.n, dtype=torch.int32, device="cuda") for f in forms}
        ms = {f: [] for f in forms}
        tot = int(w.lens.astype(np.uint64).sum())
        for r in range(rounds):
            for f in forms:
                os.environ["ICRC_AB_LONG_SELF"] = "1" if f[0] in "sk" else f
                os.environ["ICRC_AB_SELF_GRID"] = f[1:] if f.startswith("s") else "1"
                if f.startswith("k"):  # "k<e>": in place, oct wave skew e (ICRC_AB_SKEW_OCT)
                    os.environ["ICRC_AB_SKEW_OCT"] = f[1:]
                else:
                    os.environ.pop("ICRC_AB_SKEW_OCT", None)
                fn = lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), w.n,  # noqa: E731
                                               out[f].data_ptr(), False, 0, s)
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                ms[f].append(a.elapsed_time(e) / 10)
        same = all(bool(torch.equal(out[forms[0]], out[f])) for f in forms)
        for f in forms:
            m = float(np.median(ms[f]))
            print(json.dumps({"batch": name, "form": f, "ms_median": round(m, 4),
                              "ms_all": [round(x, 4) for x in ms[f]], "frac_of_8TB/s": round(tot / (m * 1e-3) / 8e12, 4),
                              "results_identical": same}), flush=True)
        del b, off, ln, out
        torch.cuda.empty_cache()
    os.environ.pop("ICRC_AB_LONG_SELF", None)
    os.environ.pop("ICRC_AB_SELF_GRID", None)
    os.environ.pop("ICRC_AB_SKEW_OCT", None)


if __name__ == "__main__":
    main()
