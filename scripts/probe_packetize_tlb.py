"""probe_packetize_tlb.py — the packetizer leg of bench.py --extra (fused_send_receive) twice in
one process: first on a fresh caching allocator, then after the other --extra legs' allocations
and torch.cuda.empty_cache() (the placement under which probe_packetize_alloc.py read 1.17 ms
instead of 1.37).  Run under rocprofv3 --pmc with address-translation counters to see whether
the two placements differ in UTCL1 misses.  PK_STEPS launches per leg (default 10)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def main():
    args = bench.ARGS = bench.parse(["--steps", os.environ.get("PK_STEPS", "10"), "--warmup", "2"])
    eng = icrc_amd.Engine(0)
    stream = torch.cuda.current_stream().cuda_stream
    r1 = bench.fused_send_receive(eng, stream, args, 1)
    for w in (workloads.write_middle_stream(args.packets), workloads.write_middle_stream(args.packets, stride=4224),
              workloads.mixed_mtu_stream(4 << 20), workloads.write_message(16 << 20, 4096)):
        d = workloads.synthesize(eng, w, stream=stream)
        torch.cuda.synchronize()
        del d
    torch.cuda.empty_cache()
    r2 = bench.fused_send_receive(eng, stream, args, 1)
    print(json.dumps({"fresh_packetize_ms": r1["packetize_send"]["kernel_ms"], "fresh_rx_ms": r1["rx_verify_parse"]["kernel_ms"],
                      "after_empty_cache_packetize_ms": r2["packetize_send"]["kernel_ms"],
                      "after_empty_cache_rx_ms": r2["rx_verify_parse"]["kernel_ms"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
