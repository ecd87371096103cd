#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_pmc.sh).

Per kernel name: mean counter value per dispatch (KB, summed over the counter's instances),
converted to bytes.  For membench dispatches the algorithmic read bytes are known
(1 Mi x 4156 B, or L-4 per packet for the row patterns), which gives the FETCH_SIZE
calibration factor for these access widths (MI355X_MICROARCH.md: FETCH_SIZE under-reports
wide streaming reads by 2x on gfx950; other widths must be calibrated)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N, L = 1 << 20, 4156


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
            per[names[k]].append(v)
    return per


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    res = {}
    for src in ("bench", "mem"):
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            per = load(os.path.join(out, f"pmc_{src}_{c}", "**", "*.csv"))
            for name, vals in per.items():
                short = name.split("(")[0][-80:]
                d = res.setdefault(src, {}).setdefault(short, {})
                d[c + "_KB_mean"] = sum(vals) / len(vals)
                d[c + "_KB_min"] = min(vals)
                d["dispatches_" + c] = len(vals)
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
        if "icrc_batch_kernel" in name and "FETCH_SIZE_KB_mean" in d:
            f = [v for k, v in factors.items() if "rows_chunk" in k or "rows_dword" in k]
            corr = sum(f) / len(f) if f else 2.0
            fetch = d["FETCH_SIZE_KB_mean"] * 1024.0 * corr
            write = d.get("WRITE_SIZE_KB_mean", 0.0) * 1024.0
            res["icrc_traffic_per_launch"] = {
                "kernel": name, "fetch_bytes_corrected": fetch, "write_bytes": write,
                "traffic_bytes": fetch + write, "algorithmic_bytes": N * L,
                "ratio_to_algorithmic": (fetch + write) / (N * L), "fetch_correction": corr}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
