#!/usr/bin/env python3
"""Run one workload a few times with the default dispatch (for rocprofv3 --pmc / --stats).

usage: run_workload.py {c1,c2,c3,s316} [launches] [variant]   (s316: 4 Mi strided 316-byte packets)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = icrc_amd.Engine(0)
    if len(sys.argv) > 3:
        eng.set_variant(int(sys.argv[3]))
    s = torch.cuda.current_stream().cuda_stream
    if which in ("c1", "s316"):
        w = workloads.write_middle_stream(1 << 20) if which == "c1" else workloads.write_middle_stream(1 << 22, pmtu=256)
        L = int(w.lens[0])
        b = workloads.synthesize(eng, w, stream=s)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        fn = lambda: eng.compute_strided(b.data_ptr(), L, L, w.n, out.data_ptr(), False, s)  # noqa: E731
    else:
        w = workloads.mixed_mtu_stream(4 << 20) if which == "c2" else workloads.write_message(16 << 20, 4096)
        b = workloads.synthesize(eng, w, stream=s)
        o = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        fn = lambda: eng.compute_batch(b.data_ptr(), o.data_ptr(), ln.data_ptr(), w.n, out.data_ptr(), False, 0, s)  # noqa: E731
    for _ in range(launches):
        fn()
    torch.cuda.synchronize()
    print(f"{which}: {launches} launches done", flush=True)


if __name__ == "__main__":
    main()
