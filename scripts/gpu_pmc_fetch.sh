#!/bin/bash
# FETCH_SIZE (one rocprofv3 --pmc pass each) over scripts/run_workload.py workloads: WL is a list
# of "workload[:variant]".  Output: gpurun_out/pmc_fetch_summary.txt (KB per dispatch per kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
for item in ${WL:-c2 c2nr c2s c2k c2m c2:140}; do
  w=${item%%:*}; v=""; [ "$item" != "$w" ] && v=${item#*:}
  tag=$(echo "$item" | tr ':' '_')
  for C in ${CTRS:-FETCH_SIZE}; do
    rm -rf $OUT/pmcf_${tag}_$C
    timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmcf_${tag}_$C -o pmc --output-format csv -- \
      python3 scripts/run_workload.py $w 3 $v > $OUT/pmcf_${tag}_$C.log 2>&1; rc=$?
    tail -1 $OUT/pmcf_${tag}_$C.log; fatal $rc "pmc $item $C"
  done
done
python3 - <<'PY' | tee $OUT/pmc_fetch_summary.txt
import csv, glob, collections, os
for d in sorted(glob.glob("gpurun_out/pmcf_*")):
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "")
            k = k.split("(icrc::BatchParams")[0].split("(BatchParams")[0][:80]
            acc[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id"))
    for (k, c), v in sorted(acc.items()):
        if "icrc" in k and "synth" not in k:
            print(os.path.basename(d), "|", k, "|", c, round(v / max(1, len(disp[(k, c)])), 1), "KB/dispatch")
PY
echo "== done"
