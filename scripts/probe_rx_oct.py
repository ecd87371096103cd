#!/usr/bin/env python3
"""A/B: the strided receive (icrc_rx_parse_device) on 4 Mi x 316 B (and 1 Mi x 1084 B) with the
two passes (ICRC_AB_RX_OCT=0), the one pass (1) and its cuts (2 no record writes, 3 no block decode
/ stores, 4 neither: the 16-copy verify alone, 5 the decode with its stores out of range; 6 16-byte
descriptor stores, 7 non-temporal ones, 8 both); plus the
verify dispatch alone ("verify").  One process, alternating rounds; one JSON line per (shape, form):
median ms of ROUNDS x 10 calls (event-timed, the whole call)."""
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
    forms = os.environ.get("FORMS", "0,1,2,3,4,5,verify").split(",")
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    shapes = [("4Mi x 316 B", workloads.write_middle_stream(4 << 20, pmtu=256), False),
              ("1Mi x 1084 B", workloads.write_middle_stream(1 << 20, pmtu=1024), False)]
    if os.environ.get("RAGGED"):  # the same through (offset, length) arrays, and configs[2]
        shapes = [("4Mi x 316 B ragged", workloads.write_middle_stream(4 << 20, pmtu=256), True),
                  ("C2 mixed MTU", workloads.mixed_mtu_stream(4 << 20), True),
                  ("786K x 4156 B ragged", workloads.write_middle_stream(786432), True)]
    for name, w, ragged in shapes:
        L = int(w.lens[0])
        b = workloads.synthesize(eng, w, stream=s)
        d_off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
        d_len = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
        tmp = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        eng.compute_batch(b.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n, tmp.data_ptr(), True, 0, s)
        desc = torch.empty(w.n * 72, dtype=torch.uint8, device="cuda")
        ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
        ms = {f: [] for f in forms}
        same = {}
        for r in range(rounds):
            for f in forms:
                if f == "verify":
                    if ragged:
                        fn = lambda: eng.verify_batch(b.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n,  # noqa: E731
                                                      ok.data_ptr(), False, 0, s)
                    else:
                        fn = lambda: eng.verify_strided(b.data_ptr(), L, L, w.n, ok.data_ptr(), False, s)  # noqa: E731
                else:
                    os.environ["ICRC_AB_RX_OCT"] = f
                    if ragged:
                        fn = lambda: eng.rx_parse(b.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), w.n,  # noqa: E731
                                                  desc.data_ptr(), ok.data_ptr(), stream=s)
                    else:
                        fn = lambda: eng.rx_parse(b.data_ptr(), 0, 0, w.n, desc.data_ptr(), ok.data_ptr(),  # noqa: E731
                                                  stride=L, length=L, stream=s)
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
                if r == 0 and f != "verify":
                    if f == forms[0]:
                        ref = desc.clone()
                    same[f] = bool(torch.equal(desc, ref))
        tot = int(w.lens.astype(np.uint64).sum())
        for f in forms:
            m = float(np.median(ms[f]))
            print(json.dumps({"shape": name, "form": f, "ms_median": round(m, 4), "ms_all": [round(x, 4) for x in ms[f]],
                              "packet_GB/s": round(tot / (m * 1e-3) / 1e9, 1),
                              "desc_identical_to_first_form": same.get(f)}), flush=True)
        del b, tmp, desc, ok, d_off, d_len
        torch.cuda.empty_cache()
    os.environ.pop("ICRC_AB_RX_OCT", None)


if __name__ == "__main__":
    main()
