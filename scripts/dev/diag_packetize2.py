"""Diagnostic: single-message packetizer cases; prints the packet words that differ from the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "open-rdma-driver_amd")]
import numpy as np  # noqa: E402

import torch  # noqa: E402

torch.cuda.init()
import icrc_amd  # noqa: E402
import oracle  # noqa: E402
import test_gpu_parity as t  # noqa: E402

eng = icrc_amd.Engine(0)
rng = np.random.default_rng(5)
src = rng.integers(1, 256, 1 << 16, dtype=np.uint8)
for total, lva, pmtu, poff, stride in [(3880, 216, 4096, 0, 4160), (3880, 0, 4096, 0, 4160), (4096, 0, 4096, 0, 4160),
                                        (716, 0, 4096, 0, 4160), (260, 0, 4096, 0, 4160), (716, 0, 4096, 64, 4160),
                                        (2400, 0, 4096, 0, 4160), (8000, 0, 4096, 0, 4160), (716, 0, 4096, 0, 8192)]:
    msgs = icrc_amd.write_messages([dict(local_va=lva, remote_va=0, payload_offset=poff, total_len=total, pmtu=pmtu,
                                         rkey=1, dqpn=1, psn=0, msn=0, dst_ip=1, kind=0)], slot_stride=stride)
    wb = int(msgs["npackets"][0]) * stride
    want, wl, wi = oracle.send_messages(src, msgs, wb)
    got, gl, gi = t.run_packetize(eng, src, msgs, wb)
    for s in range(int(msgs["npackets"][0])):
        L = int(wl[s])
        a = got[s * stride: s * stride + L - 4].view("<u4")
        b = want[s * stride: s * stride + L - 4].view("<u4")
        bad = np.nonzero(a != b)[0]
        self_icrc = oracle.compute_icrc(got[s * stride: s * stride + L])
        print(f"selfcrc {'ok' if self_icrc == gi[s] else 'BAD'} total {total} lva {lva} poff {poff} stride {stride} seg {s} L {L} gl {gl[s]} icrc {'ok' if gi[s] == wi[s] else 'BAD'} "
              f"bad words {bad.tolist()[:10]} got {[hex(x) for x in a[bad[:4]]]} want {[hex(x) for x in b[bad[:4]]]}")
