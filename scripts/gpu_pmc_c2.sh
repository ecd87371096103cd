#!/bin/bash
# C2 (mixed MTU) HBM traffic and SQ counters on the DEFAULT one-launch hybrid kernel, plus the
# FETCH_SIZE calibration for the short-packet access shape (8 packets per wave, 32-B dword rows,
# default cache policy) on scripts/shortbench.hip's known byte counts.  One rocprofv3 --pmc pass
# per counter group.  Output: gpurun_out/pmc_c2_summary.txt (per kernel, per dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
run() {  # $1 tag, $2 counters, rest: command
  local tag=$1 ctr=$2; shift 2
  rm -rf $OUT/pmcc2_$tag
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $OUT/pmcc2_$tag -o pmc --output-format csv -- "$@" > $OUT/pmcc2_$tag.log 2>&1
  local rc=$?; tail -1 $OUT/pmcc2_$tag.log; fatal $rc "pmc $tag"
}
run sb_fetch FETCH_SIZE ./scripts/_build/shortbench
for W in c2 s316; do
  run ${W}_fetch FETCH_SIZE python3 scripts/run_workload.py $W 3
  run ${W}_write WRITE_SIZE python3 scripts/run_workload.py $W 3
done
run c2_sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  python3 scripts/run_workload.py c2 3
run c2_sq2 "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
  python3 scripts/run_workload.py c2 3
python3 - <<'PY' | tee $OUT/pmc_c2_summary.txt
import csv, glob, collections
for tag in ("sb_fetch", "c2_fetch", "c2_write", "s316_fetch", "s316_write", "c2_sq1", "c2_sq2"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for path in glob.glob(f"gpurun_out/pmcc2_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "")
            k = k.split("(icrc::BatchParams")[0].split("(BatchParams")[0].split("(unsigned char")[0][:90]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r.get("Dispatch_Id"))
    for k, d in sorted(acc.items()):
        if "short_rows" in k or "icrc" in k:
            nd = max(1, len(disp[k]))
            print(tag, "|", k, "| dispatches", nd, "|", {c: round(v / nd, 1) for c, v in sorted(d.items())})
PY
echo "== done"
