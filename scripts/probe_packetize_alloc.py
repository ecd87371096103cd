"""probe_packetize_alloc.py — why bench.py --extra once read the packetizer at 1.76 ms when rocprof
of the same build read 1.37 ms.  One process, the bench's own
fused_send_receive leg timed under different allocator histories:

  fresh        the leg first, on a fresh caching allocator
  after_churn  after the same allocate / free sequence the --extra legs before it run (C1 batch,
               padded C1, mixed MTU, 16 MiB message), no empty_cache
  empty_cache  the same churn, then torch.cuda.empty_cache() before the leg
  repeat       the leg again right after (its buffers come back from the cache)

Prints one JSON line per condition (kernel ms of packetize_send and rx_verify_parse, plus the
device addresses of the leg's d_src / d_wire to show placement).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def churn(eng, stream, n):
    for w in (workloads.write_middle_stream(n), workloads.write_middle_stream(n, stride=4224),
              workloads.mixed_mtu_stream(4 << 20), workloads.write_message(16 << 20, 4096)):
        d = workloads.synthesize(eng, w, stream=stream)
        o = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        del d, o


def main():
    args = bench.ARGS = bench.parse(["--steps", os.environ.get("PK_STEPS", "50"), "--warmup", "10"])
    eng = icrc_amd.Engine(0)
    stream = torch.cuda.current_stream().cuda_stream
    order = os.environ.get("ORDER", "fresh,after_churn,empty_cache,repeat").split(",")
    for cond in order:
        if cond == "after_churn":
            churn(eng, stream, args.packets)
        elif cond == "empty_cache":
            churn(eng, stream, args.packets)
            torch.cuda.empty_cache()
        r = bench.fused_send_receive(eng, stream, args, 1)
        st = torch.cuda.memory_stats()
        print(json.dumps({"condition": cond, "packetize_ms": r["packetize_send"]["kernel_ms"],
                          "rx_ms": r.get("rx_verify_parse", {}).get("kernel_ms"),
                          "reserved_GiB": round(st["reserved_bytes.all.current"] / 2**30, 2),
                          "segments": st["segment.all.current"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
