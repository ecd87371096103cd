"""probe_packetize_alloc.py — why bench.py --extra once read the packetizer at 1.76 ms when rocprof
of the same build read 1.37 ms, and why a later probe read 1.17 ms after
torch.cuda.empty_cache().  One process; the bench's fused-send workload (192 x 16 MiB WRITE
messages -> 786 K x 4156-B packets, 3 GiB payload -> 3.2 GiB wire) timed with its buffers placed
in different ways:

  separate     d_src and d_wire as two torch allocations (what bench.py does)
  one_segment  both as slices of ONE allocation (src first, wire after it)
  swapped      both slices of one allocation, wire first
  after_free   separate, after the first pair was freed and the cache emptied

Each condition also times the receive parse over its wire buffer.  Prints one JSON line per
condition with the kernel ms and the buffers' device addresses.  Set PYTORCH_HIP_ALLOC_CONF in
the environment to compare allocator modes across processes.
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


def workload(npk_max):
    nmsg = max(1, npk_max // 4096)
    specs = [dict(local_va=0x7F0000000000 + i * MSG, remote_va=0x7E0000000000 + i * MSG, payload_offset=i * MSG,
                  total_len=MSG, pmtu=PMTU, rkey=0x2000003, dqpn=2 + i, psn=0, msn=i & 0xFFFF, dst_ip=0xC0A80003,
                  kind=0) for i in range(nmsg)]
    msgs = icrc_amd.write_messages(specs, slot_stride=SLOT)
    return nmsg, msgs, int(msgs["npackets"].sum())


def fill(d_src):
    g = torch.Generator(device="cuda").manual_seed(5)
    for c0 in range(0, d_src.numel(), 1 << 30):
        c1 = min(d_src.numel(), c0 + (1 << 30))
        d_src[c0:c1] = torch.randint(0, 256, (c1 - c0,), dtype=torch.uint8, device="cuda", generator=g)


def measure(eng, stream, args, nmsg, msgs, npk, d_src, d_wire):
    d_msgs = bench.dev(msgs.view(np.uint8))
    d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
    d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
    fill(d_src)
    torch.cuda.synchronize()
    src_bytes, wire_bytes = d_src.numel(), d_wire.numel()

    def send():
        eng.packetize(d_src.data_ptr(), src_bytes, d_msgs.data_ptr(), nmsg, npk, d_wire.data_ptr(), wire_bytes,
                      d_len.data_ptr(), d_icrc.data_ptr(), stream)

    _, pk_ms = bench.time_kernel(send, args.steps, args.warmup, 1)
    ok = bool((d_len == SLOT).all().item())
    d_off = torch.arange(npk, dtype=torch.int64, device="cuda") * SLOT
    d_desc = torch.empty(npk * 72, dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(npk, dtype=torch.uint8, device="cuda")

    def recv():
        eng.rx_parse(d_wire.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), npk, d_desc.data_ptr(), d_ok.data_ptr(),
                     stream=stream)

    _, rx_ms = bench.time_kernel(recv, args.steps, args.warmup, 1)
    ok = ok and bool((d_ok == 1).all().item())
    return pk_ms, rx_ms, ok


def main():
    args = bench.ARGS = bench.parse(["--steps", os.environ.get("PK_STEPS", "50"), "--warmup", "10"])
    eng = icrc_amd.Engine(0)
    stream = torch.cuda.current_stream().cuda_stream
    nmsg, msgs, npk = workload(3 << 18)
    src_bytes, wire_bytes = nmsg * MSG, npk * SLOT
    order = os.environ.get("ORDER", "separate,one_segment,swapped,after_free,separate").split(",")
    for cond in order:
        if cond in ("separate", "after_free"):
            if cond == "after_free":
                torch.cuda.empty_cache()
            d_src = torch.empty(src_bytes, dtype=torch.uint8, device="cuda")
            d_wire = torch.empty(wire_bytes, dtype=torch.uint8, device="cuda")
            keep = (d_src, d_wire)
        else:
            big = torch.empty(src_bytes + wire_bytes, dtype=torch.uint8, device="cuda")
            if cond == "one_segment":
                d_src, d_wire = big[:src_bytes], big[src_bytes:]
            else:
                d_wire, d_src = big[:wire_bytes], big[wire_bytes:]
            keep = (big,)
        pk_ms, rx_ms, ok = measure(eng, stream, args, nmsg, msgs, npk, d_src, d_wire)
        print(json.dumps({"condition": cond, "alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", ""),
                          "packetize_ms": round(pk_ms, 4), "rx_ms": round(rx_ms, 4), "ok": ok,
                          "src": hex(d_src.data_ptr()), "wire": hex(d_wire.data_ptr()),
                          "reserved_GiB": round(torch.cuda.memory_reserved() / 2**30, 2)}), flush=True)
        del d_src, d_wire, keep
    eng.close()


if __name__ == "__main__":
    main()
