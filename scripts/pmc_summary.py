#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_check.sh PMC=1).

Per kernel: mean counter value per dispatch (KB, summed over the counter's instances), in bytes.
For the membench dispatches the algorithmic read bytes are known (1 Mi x 4156 B, or L-4 per
packet for the row patterns), which calibrates FETCH_SIZE for these access widths on gfx950
(MI355X_MICROARCH.md, HBM section: FETCH_SIZE reports 1/2 of the bytes of a wide streaming read;
other widths must be calibrated on a known byte count).

The `icrc_traffic_per_launch` block is what bench.py reports as roofline.traffic: the ICRC
compute kernel's corrected FETCH bytes + WRITE bytes per launch over the C1 batch."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

N, L = 1 << 20, 4156
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import C2_SOURCES, kernel_source_hash  # noqa: E402  (sha of the kernel sources a record describes)

# FETCH_SIZE per counted byte for the oct kernel's access shape (8 packets per wave, 32-byte dword
# rows, default policy), calibrated on scripts/shortbench.hip's known byte counts: x1.983 on 316-B
# and x1.958 on 1084-B packets (profiles/r03_pmc_c2.txt); configs[2] is 88 % 316-B-class packets.
OCT_FETCH_CORRECTION = 1.98


def short(name):
    """'void icrc::(anonymous namespace)::icrc_batch_kernel<0, 1, 1, 8>(icrc::BatchParams)' ->
    'icrc_batch_kernel<0, 1, 1, 8>'"""
    head = re.sub(r"^void ", "", name.replace("(anonymous namespace)", "anon").split("(")[0])
    base, sep, tmpl = head.partition("<")
    return base.split("::")[-1] + sep + tmpl


def load(pattern):
    per = defaultdict(list)
    for path in glob.glob(pattern, recursive=True):
        if not path.endswith("counter_collection.csv"):
            continue
        with open(path) as f:
            rows = list(csv.DictReader(f))
        acc = defaultdict(float)
        names = {}
        for r in rows:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            acc[key] += float(r.get("Counter_Value", 0) or 0)
            names[key] = r.get("Kernel_Name", "?")
        for k, v in acc.items():
            per[short(names[k])].append(v)
    return per


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    res = {}
    for src in ("bench", "mem"):
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            per = load(os.path.join(out, f"pmc_{src}_{c}", "**", "*.csv"))
            for name, vals in per.items():
                d = res.setdefault(src, {}).setdefault(name, {})
                d[c + "_KB_mean"] = sum(vals) / len(vals)
                d[c + "_KB_min"] = min(vals)
                d["dispatches_" + c] = len(vals)
    for src in ("packetize",):
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            per = load(os.path.join(out, f"pmc_{src}_{c}", "**", "*.csv"))
            for name, vals in per.items():
                d = res.setdefault(src, {}).setdefault(name, {})
                d[c + "_KB_mean"] = sum(vals) / len(vals)
                d[c + "_KB_min"] = min(vals)
    mem = res.get("mem", {})
    known = {"flat_x4": N * L, "rows_dword": N * (L - 4), "rows_x4": N * (L - 4), "rows_chunk": N * (L - 4)}
    factors = {}
    for name, d in mem.items():
        for k, b in known.items():
            if k in name and "FETCH_SIZE_KB_min" in d:
                factors[name] = b / (d["FETCH_SIZE_KB_min"] * 1024.0)
    res["fetch_calibration_bytes_per_counted_byte"] = factors
    bench = res.get("bench", {})
    for name, d in bench.items():
        # the default C1 kernel only (variant 16: S = 2, D = 1, nt loads, TABLE = false); bench.py
        # also launches its loads-only build (variant 19, ABL 9) for the achievable denominator and
        # the small-batch form (TABLE = true: configs[3]'s 4096-packet round trip)
        if name == "icrc_batch_kernel<0, 2, 1, icrc::anon::Ring<2, true>, false>" and "FETCH_SIZE_KB_mean" in d:
            # the kernel's own shape (256-B dword rows per wave) is membench's rows_chunk / rows_dword
            f = [v for k, v in factors.items() if "rows_chunk" in k or "rows_dword" in k]
            corr = sum(f) / len(f) if f else 2.0
            fetch = d["FETCH_SIZE_KB_mean"] * 1024.0 * corr
            write = d.get("WRITE_SIZE_KB_mean", 0.0) * 1024.0
            alg = N * L
            res["icrc_traffic_per_launch"] = {
                "kernel": name, "packets": N, "packet_bytes": L, "source_hash": kernel_source_hash(),
                "fetch_bytes_counted": d["FETCH_SIZE_KB_mean"] * 1024.0,
                "fetch_correction": round(corr, 4), "fetch_bytes_corrected": round(fetch),
                "write_bytes": round(write), "traffic_bytes": round(fetch + write),
                "algorithmic_bytes": alg, "ratio_to_algorithmic": round((fetch + write) / alg, 4)}
    # configs[2]: the default one-launch hybrid kernel (compute, no trailer, dense / compacting long
    # walk by density; since round 5 each workgroup walks its own range's long packets:
    # icrc_hybrid_self_kernel) over the 4 Mi mixed-MTU batch of bench.py's c2 leg
    for name, d in bench.items():
        if (name.startswith("icrc_hybrid_self_kernel<0, false, false") or name.startswith("icrc_hybrid_kernel<0, false, false")) \
                and "FETCH_SIZE_KB_mean" in d:
            sys.path.insert(0, os.path.join(ROOT, "open-rdma-driver_amd"))
            from icrc_amd import workloads  # noqa: E402

            wm = workloads.mixed_mtu_stream(4 << 20)
            alg = int(wm.lens.astype("uint64").sum())  # L - 4 read + 4 written per packet
            fetch = d["FETCH_SIZE_KB_mean"] * 1024.0 * OCT_FETCH_CORRECTION
            write = d.get("WRITE_SIZE_KB_mean", 0.0) * 1024.0
            res["c2_traffic_per_launch"] = {
                "kernel": name, "packets": wm.n, "source_hash": kernel_source_hash(C2_SOURCES),
                "fetch_bytes_counted": d["FETCH_SIZE_KB_mean"] * 1024.0,
                "fetch_correction": OCT_FETCH_CORRECTION, "fetch_bytes_corrected": round(fetch),
                "write_bytes": round(write), "traffic_bytes": round(fetch + write),
                "algorithmic_bytes": alg, "ratio_to_algorithmic": round((fetch + write) / alg, 4),
                "note": "the (offset, length) arrays (12 B per packet) are read but not in the algorithmic bytes"}
    # the packetizer: payload read in 256-B dword rows, wire written in 256-B dword rows — the shape
    # of membench's copy_rows (known bytes: 786432 x 4096 read, 786432 x 4152 written)
    cp = {k: v for k, v in mem.items() if k.startswith("copy_rows<0, 0>")}
    npk = 786432
    for name, d in res.get("packetize", {}).items():
        if not name.startswith("icrc_packetize_kernel") or "FETCH_SIZE_KB_mean" not in d:
            continue
        fc = wc = None
        for c in cp.values():
            if c.get("FETCH_SIZE_KB_min"):
                fc = npk * 4096 / (c["FETCH_SIZE_KB_min"] * 1024.0)
            if c.get("WRITE_SIZE_KB_min"):
                wc = npk * 4152 / (c["WRITE_SIZE_KB_min"] * 1024.0)
        fetch = d["FETCH_SIZE_KB_mean"] * 1024.0 * (fc or 2.0)
        write = d.get("WRITE_SIZE_KB_mean", 0.0) * 1024.0 * (wc or 1.0)
        alg = npk * (4096 + 4156 + 8)
        res["packetize_traffic_per_launch"] = {
            "kernel": name, "packets": npk, "fetch_correction": fc, "write_correction": wc,
            "fetch_bytes_corrected": round(fetch), "write_bytes_corrected": round(write),
            "traffic_bytes": round(fetch + write), "algorithmic_bytes": alg,
            "ratio_to_algorithmic": round((fetch + write) / alg, 4)}
    print(json.dumps(res, indent=1))
    for key, fname in (("icrc_traffic_per_launch", "pmc_traffic_c1.json"), ("c2_traffic_per_launch", "pmc_traffic_c2.json")):
        if key in res:  # the records bench.py reads (copied to profiles/ as r05_pmc_traffic.json / r05_pmc_c2_traffic.json)
            with open(os.path.join(out, fname), "w") as f:
                json.dump(res[key], f, indent=1)


if __name__ == "__main__":
    main()
