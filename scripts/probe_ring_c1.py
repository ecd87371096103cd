#!/usr/bin/env python3
"""What a resident submission ring costs device batches.  C1 (compute_strided,
1 Mi x 4156 B) timed with HIP events on torch's stream: (a) with the ring's kernel ended (no host
message for 20 ms), (b) while a thread keeps the ring busy with configs[0] messages (64 x 4156 B,
compute + trailer), through the same library.  argv[1]: "product" (the default dispatch: its grid
leaves the ring's CUs out while the ring is resident) or "ab" (the A/B library; run it with
ICRC_AB_RING_AWARE=0 for the grid that counts every CU).  One JSON line per measurement."""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "product"
    L = icrc_amd.ab_library() if which == "ab" else icrc_amd.lib
    eng = icrc_amd.Engine(0, lib=L)
    s = torch.cuda.current_stream()
    w = workloads.write_middle_stream(1 << 20, 4096)
    d_buf = workloads.synthesize(eng, w, stream=s.cuda_stream)
    n, Lp = w.n, int(w.lens[0])
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    want = d_out.clone()
    eng.compute_strided(d_buf.data_ptr(), Lp, Lp, n, want.data_ptr(), False, s.cuda_stream)
    torch.cuda.synchronize()

    # configs[0] message in pinned host memory, through the library's default engine (its ring)
    msg = workloads.write_message(256 << 10, 4096)
    d_msg = workloads.synthesize(eng, msg, stream=s.cuda_stream)
    torch.cuda.synchronize()
    hm = torch.empty(d_msg.numel(), dtype=torch.uint8, pin_memory=True)
    hm.copy_(d_msg)
    hb = hm.numpy()
    off = np.ascontiguousarray(msg.off, np.uint64)
    lens = np.ascontiguousarray(msg.lens, np.uint32)
    res = np.zeros(msg.n, np.uint32)
    stop = threading.Event()
    count = [0]

    def busy():
        while not stop.is_set():
            rc = L.icrc_compute_batch(hb.ctypes.data, off.ctypes.data, lens.ctypes.data, msg.n, res.ctypes.data, 1)
            if rc != 0:
                raise RuntimeError(f"icrc_compute_batch {rc}")
            count[0] += 1

    def timed(reps=20):
        for _ in range(5):
            eng.compute_strided(d_buf.data_ptr(), Lp, Lp, n, d_out.data_ptr(), False, s.cuda_stream)
        torch.cuda.synchronize()
        per = []
        for _ in range(reps):  # one launch per event pair: the ring's state changes between launches
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.compute_strided(d_buf.data_ptr(), Lp, Lp, n, d_out.data_ptr(), False, s.cuda_stream)
            e1.record()
            e1.synchronize()
            per.append(e0.elapsed_time(e1))
        return per

    for rnd in range(3):
        time.sleep(0.02)  # the ring's kernel ends after 2 ms without a call
        alone = timed()
        th = threading.Thread(target=busy)
        th.start()
        time.sleep(0.05)
        c0, t0 = count[0], time.perf_counter()
        busy_ms = timed()
        rate = (count[0] - c0) / (time.perf_counter() - t0)
        stop.set()
        th.join()
        stop.clear()
        exact = bool(torch.equal(d_out, want))
        st = (ctypes.c_uint64 * 4)()
        h = ctypes.c_void_p()
        L.icrc_engine_default(-1, ctypes.byref(h))
        L.icrc_engine_host_stats(h, st)
        print(json.dumps({"lib": which, "aware_env": os.environ.get("ICRC_AB_RING_AWARE", "default"), "round": rnd,
                          "c1_alone_ms_median": round(float(np.median(alone)), 4),
                          "c1_ring_busy_ms_median": round(float(np.median(busy_ms)), 4),
                          "c1_ring_busy_ms_max": round(float(np.max(busy_ms)), 4),
                          "c1_ring_busy_ms_min": round(float(np.min(busy_ms)), 4),
                          "messages_per_s_during": round(rate, 1), "results_exact": exact,
                          "ring_jobs": st[0], "ring_launches": st[1]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
