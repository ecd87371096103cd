#!/usr/bin/env python3
"""configs[2]: the rows the oct kernel loads past each packet's end, counted per dispatch (VERDICT
r05 item 4: "bound the 15 % over-read").  A CPU model of run_oct's set / frame schedule on
mixed_mtu_stream(4 Mi) (csrc/icrc_oct.hip: oct_block sorts each 64-packet block by row count R;
sets are 8 consecutive sorted packets; a set runs ceil(Rmax / 10) frames of 10 row loads per lane,
rows past the set's last row re-load that row (kOctClampRows), so a lane reads Rmax DISTINCT
32-byte rows: R of its own packet's stream (the first front-padded by z = -N mod 8 words, before
the packet) and Rmax - R past its end).  Long packets (L > 1088) are the long half's (one wave per
packet, 256-B rows, end-aligned: its first row starts up to 252 B before the packet).

Prints one JSON object: packets, algorithmic bytes, bytes the model's row loads cover per
dispatch split into own rows / front padding / past the end, and the same for the long half; to
set against the measured HBM traffic (profiles/r06_pmc_c2_traffic.json).  CPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402

from icrc_amd import workloads  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else (4 << 20)
    wm = workloads.mixed_mtu_stream(n)
    L = wm.lens.astype(np.int64)
    alg = int(L.sum())
    short = L <= 1088
    N = (L - 4) // 4 + 2                 # stream words (compute: 8 FF bytes + L - 4 packet bytes)
    R = np.where(short, (N + 7) // 8, 0)  # oct rows of 8 words
    z = (-N) % 8                         # leading pad words of row 0
    nb = (n + 63) // 64
    Rp = np.zeros(nb * 64, np.int64)
    Rp[:n] = R
    Rb = Rp.reshape(nb, 64)
    past_rows = 0
    frames = 0
    for b in range(nb):
        r = np.sort(Rb[b][Rb[b] > 0])
        for k in range(0, r.size, 8):
            g = r[k:k + 8]
            past_rows += int((g.max() - g).sum())
            frames += int(-(-g.max() // 10))
    own_bytes = int(32 * R.sum())
    pad_bytes = int(4 * z[short].sum())
    past_bytes = 32 * past_rows
    # long half: 64-word rows end-aligned to the stream; row 0 starts 4 * (-N mod 64) bytes early
    zl = (-N[~short]) % 64
    long_rows = int(((N[~short] + 63) // 64).sum())
    out = {
        "packets": n, "algorithmic_bytes": alg,
        "oct_packets": int(short.sum()), "oct_sets_frames": frames,
        "oct_row_bytes_own": own_bytes, "oct_front_pad_bytes": pad_bytes,
        "oct_rows_past_end": past_rows, "oct_bytes_past_end": past_bytes,
        "long_packets": int((~short).sum()), "long_row_bytes": 256 * long_rows,
        "long_front_pad_bytes": int(4 * zl.sum()),
        "offset_length_array_bytes": 12 * n,
        "past_end_fraction_of_algorithmic": round(past_bytes / alg, 4),
        "note": "past-end rows are the next packets' bytes, which the same wave loads in the same "
                "block: they add HBM traffic only where the line has left L2 between the two reads",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
