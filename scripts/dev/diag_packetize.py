"""Diagnostic: which packetizer packets differ from the oracle (kind, flags, segment, L) and where."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "open-rdma-driver_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
import oracle  # noqa: E402
import test_gpu_parity as t  # noqa: E402

eng = icrc_amd.Engine(0)
rng = np.random.default_rng(21)
specs, src_bytes = t._random_specs(rng, 40, True)
msgs = icrc_amd.write_messages(specs)
src = rng.integers(0, 256, src_bytes + 16, dtype=np.uint8)
wire_bytes = int(msgs["out_offset"][-1]) + int(msgs["npackets"][-1]) * int(msgs["slot_stride"][-1]) + 64
want, wl, wi = oracle.send_messages(src, msgs, wire_bytes)
got, gl, gi = t.run_packetize(eng, src, msgs, wire_bytes)
for m in msgs:
    for s in range(int(m["npackets"])):
        k = int(m["first_packet"]) + s
        o = int(m["out_offset"]) + s * int(m["slot_stride"])
        L = int(wl[k])
        bad = np.nonzero(got[o:o + L] != want[o:o + L])[0]
        if gi[k] != wi[k] or bad.size:
            print(f"pk {k} kind {m['kind']} flags {m['flags']} s {s}/{m['npackets']} L {L} gl {gl[k]} pmtu {m['pmtu']} "
                  f"lva {int(m['local_va']) % 4096} icrc {'ok' if gi[k] == wi[k] else 'BAD'} bytes bad at {bad[:12].tolist()} "
                  f"got {got[o:o + L][bad[:6]].tolist()} want {want[o:o + L][bad[:6]].tolist()}")
