#!/usr/bin/env python3
"""Receive-parse and verify rates on the C1 batch: ragged (off/len arrays) vs strided, and the
plain verify kernel, to locate the receive path's losses.  One JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    n = 1 << 20
    w = workloads.write_middle_stream(n)
    L = int(w.lens[0])
    b = workloads.synthesize(eng, w, stream=s)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_strided(b.data_ptr(), L, L, n, d_out.data_ptr(), True, s)
    off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
    desc = torch.empty(n * icrc_amd.RX_DESC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cases = {
        "rx_ragged": lambda: eng.rx_parse(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, desc.data_ptr(), ok.data_ptr(), stream=s),
        "rx_strided": lambda: eng.rx_parse(b.data_ptr(), 0, 0, n, desc.data_ptr(), ok.data_ptr(), stride=L, length=L, stream=s),
        "verify_strided": lambda: eng.verify_strided(b.data_ptr(), L, L, n, ok.data_ptr(), False, s),
        "verify_ragged": lambda: eng.verify_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, ok.data_ptr(), False, 0, s),
        "compute_ragged": lambda: eng.compute_batch(b.data_ptr(), off.data_ptr(), ln.data_ptr(), n, d_out.data_ptr(), False, 0, s),
    }
    for name, fn in cases.items():
        ms = timed(fn)
        print(json.dumps({"case": name, "ms": round(ms, 4), "GB/s": round(n * L / (ms * 1e-3) / 1e9, 1)}), flush=True)
    # A/B (interleaved rounds): hybrid split with the filtered S = 2 long kernel (-1) vs the
    # compacting walker (224), and the receive kernel's S / D variants (300-302)
    wm = workloads.mixed_mtu_stream(4 << 20)
    bm = workloads.synthesize(eng, wm, stream=s)
    moff = torch.from_numpy(np.ascontiguousarray(wm.off)).cuda()
    mln = torch.from_numpy(np.ascontiguousarray(wm.lens)).cuda()
    mout = torch.zeros(wm.n, dtype=torch.int32, device="cuda")
    mtot = int(wm.lens.astype(np.int64).sum())
    c2 = lambda: eng.compute_batch(bm.data_ptr(), moff.data_ptr(), mln.data_ptr(), wm.n, mout.data_ptr(), False, 0, s)
    ref_c2 = None
    for rnd in range(2):
        for v in (-1, 224):
            eng.set_variant(v)
            for name, fn, nb in (("verify_ragged", cases["verify_ragged"], n * L), ("compute_ragged", cases["compute_ragged"], n * L),
                                 ("c2_hybrid", c2, mtot)):
                ms = timed(fn)
                print(json.dumps({"case": f"{name}_hyb{v}", "round": rnd, "ms": round(ms, 4),
                                  "GB/s": round(nb / (ms * 1e-3) / 1e9, 1)}), flush=True)
            torch.cuda.synchronize()
            r = mout.cpu().numpy().copy()
            if ref_c2 is None:
                ref_c2 = r
            print(json.dumps({"case": f"c2_same_{v}", "ok": bool((r == ref_c2).all())}), flush=True)
        for v in (300, 301, 302):
            eng.set_variant(v)
            for name in ("rx_ragged", "rx_strided"):
                ms = timed(cases[name])
                print(json.dumps({"case": f"{name}_v{v}", "round": rnd, "ms": round(ms, 4),
                                  "GB/s": round(n * L / (ms * 1e-3) / 1e9, 1)}), flush=True)
    eng.set_variant(-1)
    # forced single-kernel variants on the ragged batch (no hybrid split): where the ragged loss is
    for v in (16, 13, 14):
        eng.set_variant(v)
        for name in ("verify_ragged", "compute_ragged"):
            ms = timed(cases[name])
            print(json.dumps({"case": f"{name}_v{v}", "ms": round(ms, 4),
                              "GB/s": round(n * L / (ms * 1e-3) / 1e9, 1)}), flush=True)
    eng.set_variant(-1)


if __name__ == "__main__":
    main()
