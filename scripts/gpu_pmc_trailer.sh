#!/bin/bash
# The trailer store's memory-side cost: C1 compute without / with the
# trailer write and verify without / with the in-place zeroing (scripts/run_workload.py c1, c1w,
# c1v, c1vz), one rocprofv3 --pmc pass per counter: WRITE_SIZE, the L2's write requests to the
# fabric by size, and the L2's own write / atomic requests.  Counters the box does not list are
# skipped (the list is written to gpurun_out/rocprof_counters.txt first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
timeout -s KILL 60 rocprofv3 -L > $OUT/rocprof_counters.txt 2>&1; fatal $? "rocprofv3 -L"
for C in ${CTRS:-WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum}; do
  base=${C%_sum}
  if ! grep -q "\b$base\b" $OUT/rocprof_counters.txt; then echo "skip $C (not listed)"; continue; fi
  for W in ${WL:-c1 c1w c1v c1vz}; do
    rm -rf $OUT/pmct_${W}_$C
    timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmct_${W}_$C -o pmc --output-format csv -- \
      python3 scripts/run_workload.py $W 3 > $OUT/pmct_${W}_$C.log 2>&1; rc=$?
    tail -1 $OUT/pmct_${W}_$C.log; fatal $rc "pmc $W $C"
  done
done
python3 - <<'PY' | tee $OUT/pmc_trailer_summary.txt
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/pmct_*")):
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "")
            k = k.split("(icrc::BatchParams")[0].split("(BatchParams")[0][:80]
            acc[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id"))
    for (k, c), v in sorted(acc.items()):
        if "icrc_batch" in k:
            print(os.path.basename(d), "|", k, "|", c, round(v / max(1, len(disp[(k, c)])), 1), "per dispatch")
PY
echo "== done"
