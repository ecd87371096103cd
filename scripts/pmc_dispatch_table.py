#!/usr/bin/env python3
"""Per-case instruction counters from one rocprofv3 --pmc run whose program launched the same
kernel `per` times per case, cases in order (scripts/probe_c2_windows.py with PMC=1).

usage: pmc_dispatch_table.py <counter_collection.csv> <kernel substring> <per> <case,case,...>
Prints one JSON line per case: each counter's mean per dispatch, and the instruction counts per
vector memory read instruction (SQ_INSTS_VALU / SALU / LDS over SQ_INSTS_VMEM_RD) with
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES."""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, sub, per, names = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4].split(",")
    by = defaultdict(dict)
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if sub in r["Kernel_Name"]:
                by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    if len(ids) != per * len(names):
        print(json.dumps({"error": f"{len(ids)} dispatches of {sub!r}, expected {per} x {len(names)}"}))
        sys.exit(1)
    for k, name in enumerate(names):
        rows = [by[i] for i in ids[k * per:(k + 1) * per]]
        mean = {c: sum(r.get(c, 0.0) for r in rows) / per for c in rows[0]}
        out = {"case": name, "dispatches": per, **{c: round(v) for c, v in sorted(mean.items())}}
        vm = mean.get("SQ_INSTS_VMEM_RD", 0.0)
        if vm:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if c in mean:
                    out[c.replace("SQ_INSTS_", "") + "_per_vmem_rd"] = round(mean[c] / vm, 3)
        if mean.get("SQ_WAVE_CYCLES"):
            out["wait_inst_any_frac"] = round(mean.get("SQ_WAIT_INST_ANY", 0.0) / mean["SQ_WAVE_CYCLES"], 4)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
