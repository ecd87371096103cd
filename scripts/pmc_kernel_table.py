#!/usr/bin/env python3
"""Counters per dispatch, averaged per kernel, from rocprofv3 --pmc runs (the request table of
scripts/gpu_r06_final.sh's REQ step).

usage: pmc_kernel_table.py <label>=<pmc directory> ... [--match SUBSTRING]
Prints "label | kernel | dispatches n | {counter: mean per dispatch in millions}" per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        k = args.index("--match")
        match = args[k + 1]
        del args[k:k + 2]
    print("# requests per dispatch (millions): CU->L2 (TCP_TCC_*_REQ) and L2->memory (TCC_EA0_*REQ); "
          "scripts/gpu_r06_final.sh REQ")
    for spec in args:
        label, d = spec.split("=", 1)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        per = defaultdict(lambda: defaultdict(dict))
        for fn in files:
            with open(fn, newline="") as f:
                for r in csv.DictReader(f):
                    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                    if match and match not in name and "icrc" not in name and "rows" not in name and "flat" not in name:
                        continue
                    if name.startswith("at::"):
                        continue
                    per[name][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for name, disp in per.items():
            cs = sorted({c for v in disp.values() for c in v})
            mean = {c: round(sum(v.get(c, 0.0) for v in disp.values()) / len(disp) / 1e6, 2) for c in cs}
            print(f"{label} | {name} | dispatches {len(disp)} | {mean}")


if __name__ == "__main__":
    main()
