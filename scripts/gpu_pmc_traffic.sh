#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 --pmc run each) over one workload of
# scripts/run_workload.py (default c2); per-kernel KB per dispatch -> gpurun_out/pmctr_<W>.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
W=${WORKLOAD:-c2}; export W
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmctr_${W}_$C
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmctr_${W}_$C -o pmc --output-format csv -- \
    python3 scripts/run_workload.py $W 3 > $OUT/pmctr_${W}_$C.log 2>&1; rc=$?
  tail -1 $OUT/pmctr_${W}_$C.log; fatal $rc "pmc $C"
done
python3 - <<'PY' | tee $OUT/pmctr_$W.txt
import csv, glob, collections, os
W = os.environ["W"]
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for path in glob.glob(f"gpurun_out/pmctr_{W}_{C}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "").split("(")[0][:80]
            acc[k] += float(r["Counter_Value"]); disp[k].add(r.get("Dispatch_Id"))
    for k, v in acc.items():
        print(W, C, k, "KB/dispatch", round(v / max(1, len(disp[k])), 1), "dispatches", len(disp[k]))
PY
echo "== done"
