"""probe_packetize_place.py — is the packetizer's 1.17-1.37 ms spread a placement
effect, and does rotating each wave's start make it immune?  One process, the A/B library (its
ICRC_AB_PK_ROT switch is read per launch): the bench's fused-send workload (192 x 16 MiB WRITE
messages -> 786 K x 4156-B packets) with d_src and d_wire as slices of ONE oversized allocation,
d_wire placed `delta` bytes after the end of d_src for a sweep of deltas (256 B .. 48 MiB), each
placement timed with the waves' chunks walked in order (rot 0) and rotated (rot 1), interleaved.
Prints one JSON line per (delta, rot): median / min kernel ms over ROUNDS x 20 launches.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import icrc_amd  # noqa: E402

PMTU, MSG = 4096, 16 << 20
SLOT = 28 + 28 + PMTU + 4


def main():
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    stream = torch.cuda.current_stream().cuda_stream
    nmsg = 192
    specs = [dict(local_va=0x7F0000000000 + i * MSG, remote_va=0x7E0000000000 + i * MSG, payload_offset=i * MSG,
                  total_len=MSG, pmtu=PMTU, rkey=0x2000003, dqpn=2 + i, psn=0, msn=i & 0xFFFF, dst_ip=0xC0A80003,
                  kind=0) for i in range(nmsg)]
    msgs = icrc_amd.write_messages(specs, slot_stride=SLOT)
    npk = int(msgs["npackets"].sum())
    src_bytes, wire_bytes = nmsg * MSG, npk * SLOT
    deltas = [int(x) for x in os.environ.get("DELTAS", "0,256,4096,65536,262144,786432,1048576,2097152,3145728,"
                                                     "8388608,25165824,50331648").split(",")]
    slack = max(deltas) + (1 << 21)
    big = torch.empty(src_bytes + wire_bytes + slack, dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    for c0 in range(0, src_bytes, 1 << 30):
        c1 = min(src_bytes, c0 + (1 << 30))
        big[c0:c1] = torch.randint(0, 256, (c1 - c0,), dtype=torch.uint8, device="cuda", generator=g)
    d_msgs = bench.dev(msgs.view(np.uint8))
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    rounds = int(os.environ.get("ROUNDS", "3"))
    ref = None
    for delta in deltas:
        wire = big.data_ptr() + src_bytes + delta
        times = {0: [], 1: []}
        for _ in range(rounds):
            for rot in (0, 1):
                os.environ["ICRC_AB_PK_ROT"] = str(rot)

                def send():
                    eng.packetize(big.data_ptr(), src_bytes, d_msgs.data_ptr(), nmsg, npk, wire, wire_bytes,
                                  d_len.data_ptr(), d_icrc.data_ptr(), stream)

                send()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    send()
                e1.record()
                torch.cuda.synchronize()
                times[rot].append(e0.elapsed_time(e1) / 20)
                got = d_icrc.cpu().numpy()
                if ref is None:
                    ref = got.copy()
                assert np.array_equal(got, ref), f"ICRCs differ at delta {delta} rot {rot}"
                assert bool((d_len == SLOT).all().item())
        for rot in (0, 1):
            ts = times[rot]
            print(json.dumps({"delta": delta, "rot": rot, "ms_median": round(float(np.median(ts)), 4),
                              "ms_min": round(min(ts), 4), "src": hex(big.data_ptr()), "wire": hex(wire),
                              "TB/s": round(npk * (4096 + 4156 + 8) / (float(np.median(ts)) * 1e-3) / 1e12, 3)}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
