#!/bin/bash
# Address-translation counters for scripts/probe_packetize_tlb.py (one rocprofv3 --pmc pass per
# counter); per-dispatch values of the packetize and receive kernels, in dispatch order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
timeout -k 10 300 python3 scripts/probe_packetize_tlb.py > $OUT/tlb_plain.json 2> $OUT/tlb_plain.err; rc=$?
cat $OUT/tlb_plain.json; fatal $rc plain
for C in ${CTRS:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum TCP_PENDING_STALL_CYCLES_sum}; do
  rm -rf $OUT/pmctlb_$C
  timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/pmctlb_$C -o pmc --output-format csv -- \
    python3 scripts/probe_packetize_tlb.py > $OUT/pmctlb_$C.log 2>&1; rc=$?
  tail -1 $OUT/pmctlb_$C.log; fatal $rc "pmc $C"
done
python3 - <<'PY' | tee $OUT/pmc_tlb_summary.txt
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/pmctlb_*")):
    if not os.path.isdir(d):
        continue
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if "packetize" in k or "rx_desc" in k:
                rows["packetize" if "packetize" in k else "rx_desc"][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for k, dd in rows.items():
        ids = sorted(dd)
        vals = [dd[i] for i in ids]
        h = len(vals) // 2
        print(os.path.basename(d), k, "dispatches", len(vals), "first half mean", round(sum(vals[:h]) / max(1, h)),
              "second half mean", round(sum(vals[h:]) / max(1, len(vals) - h)))
PY
echo "== done"
