#!/usr/bin/env python3
"""Does the receive parse's descriptor pass read the header lines from the Infinity Cache when it
runs right after the verify pass of the same packets?  4 Mi ragged 316-byte packets (1.33 GB):
rx_parse over the whole batch, then over 4 / 8 / 16 consecutive chunks (each chunk's verify pass
and descriptor pass back to back).  Run under `rocprofv3 --kernel-trace` (scripts/gpu_rx_chunks.sh)
to sum each pass's kernel durations per chunking; the event time per call sequence is printed here."""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    w = workloads.write_middle_stream(1 << 22, pmtu=256)
    b = workloads.synthesize(eng, w, stream=s)
    off = torch.from_numpy(np.ascontiguousarray(w.off)).cuda()
    ln = torch.from_numpy(np.ascontiguousarray(w.lens)).cuda()
    ok = torch.zeros(w.n, dtype=torch.uint8, device="cuda")
    dsz = icrc_amd.RX_DESC_DTYPE.itemsize
    d = torch.zeros(w.n * dsz, dtype=torch.uint8, device="cuda")
    for chunks in (1, 4, 8, 16, 1):
        per = w.n // chunks

        def run():
            for c in range(chunks):
                lo = c * per
                eng.rx_parse(b.data_ptr(), off.data_ptr() + 8 * lo, ln.data_ptr() + 4 * lo, per,
                             d.data_ptr() + dsz * lo, ok.data_ptr() + lo, stream=s)
        run()
        torch.cuda.synchronize()
        ref = d.clone() if chunks == 1 else None
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            run()
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"chunks": chunks, "packets": w.n, "ms_per_batch": round(a.elapsed_time(e) / reps, 4)}), flush=True)
        if ref is not None:
            ref0 = ref
        else:
            assert torch.equal(d, ref0), "chunked parse differs"


if __name__ == "__main__":
    main()
