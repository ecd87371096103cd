#!/usr/bin/env python3
"""Staged large-size checks of the fused receive and send kernels (one process, sync + report
after every stage so a fault names its stage).  Sizes: C1 (1 Mi x 4156 B)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def say(msg):
    print(msg, flush=True)


def main():
    import icrc_amd
    from icrc_amd import workloads

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    eng = icrc_amd.Engine(0)
    s = torch.cuda.current_stream().cuda_stream
    w = workloads.write_middle_stream(n, 4096)
    L = int(w.lens[0])
    d_buf = workloads.synthesize(eng, w, stream=s)
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_strided(d_buf.data_ptr(), L, L, n, d_out.data_ptr(), True, s)
    torch.cuda.synchronize()
    say(f"stage 1 compute+trailer ok: n={n}")

    d_desc = torch.zeros(n * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    eng.rx_parse(d_buf.data_ptr(), 0, 0, n, d_desc.data_ptr(), d_ok.data_ptr(), stride=L, length=L, stream=s)
    torch.cuda.synchronize()
    say(f"stage 2 rx strided ok: all_ok={bool((d_ok == 1).all().item())}")

    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * L
    d_len = torch.full((n,), L, dtype=torch.int32, device="cuda")
    d_ok.zero_()
    eng.rx_parse(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_desc.data_ptr(), d_ok.data_ptr(), stream=s)
    torch.cuda.synchronize()
    say(f"stage 3 rx ragged ok: all_ok={bool((d_ok == 1).all().item())}")
    del d_buf, d_desc, d_ok, d_off, d_len, d_out
    torch.cuda.empty_cache()

    nmsg = max(1, n // 4096)
    msg_bytes = 16 << 20
    specs = [dict(local_va=0x7F0000000000 + i * msg_bytes, remote_va=0x7E0000000000 + i * msg_bytes,
                  payload_offset=i * msg_bytes, total_len=msg_bytes, pmtu=4096, rkey=3, dqpn=2 + i, psn=0,
                  msn=i & 0xFFFF, dst_ip=0xC0A80003, kind=0) for i in range(nmsg)]
    msgs = icrc_amd.write_messages(specs, slot_stride=L)
    npk = int(msgs["npackets"].sum())
    src_bytes = nmsg * msg_bytes
    d_src = torch.empty(src_bytes, dtype=torch.uint8, device="cuda")
    for c0 in range(0, src_bytes, 1 << 30):
        c1 = min(src_bytes, c0 + (1 << 30))
        d_src[c0:c1] = (torch.arange(c1 - c0, device="cuda", dtype=torch.int64) % 251).to(torch.uint8)
    torch.cuda.synchronize()
    say(f"stage 4 source ready: {src_bytes} bytes")
    d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).cuda()
    d_wire = torch.zeros(npk * L, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    eng.packetize(d_src.data_ptr(), src_bytes, d_msgs.data_ptr(), nmsg, npk, d_wire.data_ptr(), npk * L,
                  d_len.data_ptr(), d_icrc.data_ptr(), stream=s)
    torch.cuda.synchronize()
    lens = d_len.cpu().numpy()
    say(f"stage 5 packetize ok: lengths all {L}: {bool(np.all(lens == L))}, distinct {np.unique(lens)[:8]}")
    d_off = torch.arange(npk, dtype=torch.int64, device="cuda") * L
    d_desc = torch.zeros(npk * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(npk, dtype=torch.uint8, device="cuda")
    eng.rx_parse(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_desc.data_ptr(), d_ok.data_ptr(),
                 stream=s)
    torch.cuda.synchronize()
    say(f"stage 6 rx over packetized wire ok: all_ok={bool((d_ok == 1).all().item())}")
    del d_src, d_wire, d_desc
    torch.cuda.empty_cache()
    # row-stream variants (10-12) at C1 size with offset/length arrays
    w = workloads.write_middle_stream(n, 4096)
    d_buf = workloads.synthesize(eng, w, stream=s)
    d_off = torch.arange(n, dtype=torch.int64, device="cuda") * L
    d_len = torch.full((n,), L, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out.data_ptr(), True, 0, s)
    d_ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    eng.set_variant(10)  # row stream, ragged meta blocks: compute, then verify
    d_out2 = torch.zeros(n, dtype=torch.int32, device="cuda")
    eng.compute_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_out2.data_ptr(), False, 0, s)
    torch.cuda.synchronize()
    say(f"stage 3a row-stream compute ragged ok: same={bool(torch.equal(d_out, d_out2))}")
    d_ok.zero_()
    eng.verify_batch(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, d_ok.data_ptr(), False, 0, s)
    torch.cuda.synchronize()
    say(f"stage 3b row-stream verify ragged ok: all_ok={bool((d_ok == 1).all().item())}")
    eng.set_variant(-1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
