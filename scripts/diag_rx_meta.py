#!/usr/bin/env python3
"""Meta-walk check of the fused receive kernel (ICRC_RX_DEBUG=1 path: no packet bytes are
touched; each packet's descriptor records the index, offset and length the kernel walked)."""
import os
import sys

os.environ["ICRC_RX_DEBUG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import icrc_amd

    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    L = 4156
    for n in (4096, 16384, 1 << 20):
        d_buf = torch.zeros(64, dtype=torch.uint8, device="cuda")  # never dereferenced in this mode
        for ragged in (False, True):
            d_off = torch.arange(n, dtype=torch.int64, device="cuda") * L
            d_len = torch.full((n,), L, dtype=torch.int32, device="cuda")
            d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
            if ragged:
                eng.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(), stream=s)
            else:
                eng.rx_parse(d_buf.data_ptr(), 0, 0, n, d_desc.data_ptr(), stride=L, length=L, stream=s)
            torch.cuda.synchronize()
            d = d_desc.cpu().numpy().view("<u4").reshape(n, 18)
            idx = np.arange(n, dtype=np.uint64)
            off = d[:, 4].astype(np.uint64) | (d[:, 5].astype(np.uint64) << np.uint64(32))
            bad = np.nonzero((d[:, 0] != idx) | (off != idx * np.uint64(L)) | (d[:, 6] != L) | (d[:, 17] != 1))[0]
            print(f"n={n} ragged={ragged}: bad={bad.size}", flush=True)
            for i in bad[:8]:
                print(f"  i={i}: idx={d[i, 0]} off={off[i]} (want {i * L}) L={d[i, 6]} kind={d[i, 17]}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
