"""probe_env_ab.py — A/B of an ICRC_AB_* switch of the A/B library (read per launch) on the batches
of scripts/ab_variants.py, in ONE process, interleaved rounds, results checked equal.

usage: AB_ENV=ICRC_AB_OCT_NOSKIP AB_VALUES=0,1 JOBS=C2,C2m,S316 python3 scripts/probe_env_ab.py
Prints one JSON line per (job, value): median / min of ROUNDS x 10 launches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-rdma-driver_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icrc_amd  # noqa: E402
from icrc_amd import workloads  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def main():
    env = os.environ["AB_ENV"]
    values = os.environ.get("AB_VALUES", "0,1").split(",")
    eng = icrc_amd.Engine(0, lib=icrc_amd.ab_library())
    s = torch.cuda.current_stream().cuda_stream
    kws = {"C2": {}, "C2m": dict(classes=(256, 1024)), "C2k": dict(classes=(1024,)), "C2s": dict(classes=(256,)),
           "C2nr": dict(ragged_frac=0.0)}
    jobs = {}
    for name in os.environ.get("JOBS", "C2,C2m").split(","):
        if name in ("PK", "PKc"):  # the fused send packetizer: 192 x 16 MiB WRITE -> 786 K x 4156-B packets
            # (PKc: the payload one constant byte instead of random bytes)
            MSG, SLOT = 16 << 20, 28 + 28 + 4096 + 4
            specs = [dict(local_va=0x7F0000000000 + i * MSG, remote_va=0x7E0000000000 + i * MSG, payload_offset=i * MSG,
                          total_len=MSG, pmtu=4096, rkey=0x2000003, dqpn=2 + i, psn=0, msn=i & 0xFFFF,
                          dst_ip=0xC0A80003, kind=0) for i in range(192)]
            msgs = icrc_amd.write_messages(specs, slot_stride=SLOT)
            npk = int(msgs["npackets"].sum())
            if name == "PKc":
                d_src = torch.full((192 * MSG,), 0x5A, dtype=torch.uint8, device="cuda")
            else:
                d_src = torch.randint(0, 256, (192 * MSG,), dtype=torch.uint8, device="cuda")
            d_wire = torch.empty(npk * SLOT, dtype=torch.uint8, device="cuda")
            d_msgs = dev(msgs.view(np.uint8))
            d_len = torch.zeros(npk, dtype=torch.int32, device="cuda")
            d_icrc = torch.zeros(npk, dtype=torch.int32, device="cuda")
            jobs[name] = (lambda d_src=d_src, d_wire=d_wire, d_msgs=d_msgs, d_len=d_len, d_icrc=d_icrc, npk=npk:
                          eng.packetize(d_src.data_ptr(), d_src.numel(), d_msgs.data_ptr(), 192, npk, d_wire.data_ptr(),
                                        d_wire.numel(), d_len.data_ptr(), d_icrc.data_ptr(), s),
                          npk * (4096 + 4156 + 8), d_icrc, (d_src, d_wire, d_msgs, d_len))
            continue
        if name in ("S316", "C1"):
            w = workloads.write_middle_stream(1 << 22, pmtu=256) if name == "S316" else workloads.write_middle_stream(1 << 20)
            L = int(w.lens[0])
            b = workloads.synthesize(eng, w, stream=s)
            out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
            jobs[name] = (lambda b=b, out=out, n=w.n, L=L: eng.compute_strided(b.data_ptr(), L, L, n, out.data_ptr(),
                                                                               False, s), w.n * L, out, b)
            continue
        if name == "R4K":  # 1 Mi x 4156-B packets as a ragged batch (offset / length arrays): every packet long
            w = workloads.write_middle_stream(1 << 20)
        else:
            w = workloads.mixed_mtu_stream(4 << 20, **kws[name])
        b = workloads.synthesize(eng, w, stream=s)
        o, l = dev(w.off), dev(w.lens)
        out = torch.zeros(w.n, dtype=torch.int32, device="cuda")
        jobs[name] = (lambda b=b, o=o, l=l, out=out, n=w.n: eng.compute_batch(b.data_ptr(), o.data_ptr(), l.data_ptr(),
                                                                             n, out.data_ptr(), False, 0, s),
                      int(w.lens.astype(np.uint64).sum()), out, (b, o, l))
    times = {(j, v): [] for j in jobs for v in values}
    ref = {}
    for _ in range(int(os.environ.get("ROUNDS", "5"))):
        for v in values:
            os.environ[env] = v
            for j, (fn, nb, out, _) in jobs.items():
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[(j, v)].append(e0.elapsed_time(e1) / 10)
                got = out.cpu().numpy().copy()
                ref.setdefault(j, got)
                if os.environ.get("AB_CHECK", "1") == "1":  # 0 for ablations (wrong results by design)
                    assert np.array_equal(ref[j], got), (j, v)
    for (j, v), ts in times.items():
        nb = jobs[j][1]
        med = float(np.median(ts))
        print(json.dumps({"env": env, "value": v, "workload": j, "ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                          "frac_of_8TB": round(nb / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
