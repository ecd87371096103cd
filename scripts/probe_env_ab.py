"""probe_env_ab.py — A/B of an ICRC_AB_* switch of the A/B library (read per launch) on the batches
of scripts/ab_variants.py, in ONE process, interleaved rounds, results checked equal.

usage: AB_ENV=ICRC_AB_OCT_NOSKIP AB_VALUES=0,1 JOBS=C2,C2m,S316 python3 scripts/probe_env_ab.py
Prints one JSON line per (job, value): median / min of ROUNDS x 10 launches."""
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
    env = os.environ["AB_ENV"]
    values = os.environ.get("AB_VALUES", "0,1").split(",")
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    kws = {"C2": {}, "C2m": dict(classes=(256, 1024)), "C2k": dict(classes=(1024,)), "C2s": dict(classes=(256,)),
           "C2nr": dict(ragged_frac=0.0)}
    jobs = {}
    for name in os.environ.get("JOBS", "C2,C2m").split(","):
        if name == "S316":
            w = workloads.write_middle_stream(1 << 22, pmtu=256)
            L = int(w.lens[0])
            b = workloads.synthesize(eng, w, stream=s)
            out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
            jobs[name] = (lambda b=b, out=out, n=w.n, L=L: eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(),
                                                                               False, s), w.n * L, out, b)
            continue
        w = workloads.mixed_mtu_stream(4 << 20, **kws[name])
        b = workloads.synthesize(eng, w, stream=s)
        o, l = dev(w.off), dev(w.lens)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        jobs[name] = (lambda b=b, o=o, l=l, out=out, n=w.n: eng.compute_batch(b.data_ptr(), o.data_ptr(), l.data_ptr(),
                                                                             n, out.data_ptr(), False, 0, s),
                      int(w.lens.astype(np.uint64).sum()), out, (b, o, l))
    times = {(j, v): [] for j in jobs for v in values}
    ref = {}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for v in values:
            os.environ[env] = v
            for j, (fn, nb, out, _) in jobs.items():
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, v)].append(e0.elapsed_time(e1) / 10)
                got = out.cpu().numpy().copy()
                ref.setdefault(j, got)
                assert np.array_equal(ref[j], got), (j, v)
    for (j, v), ts in times.items():
        nb = jobs[j][1]
        med = float(np.median(ts))
        print(json.dumps({"env": env, "value": v, "workload": j, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "frac_of_8TB": round(nb / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
