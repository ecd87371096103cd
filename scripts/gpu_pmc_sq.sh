#!/bin/bash
# SQ counter passes over one workload (scripts/run_workload.py), one rocprofv3 --pmc run each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
W=${WORKLOAD:-c2}; TAG=${W}_${VARIANT:-dflt}; export TAG
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  rm -rf $OUT/pmcsq_${TAG}_$i
  timeout -s KILL 120 rocprofv3 --pmc $SET -d $OUT/pmcsq_${TAG}_$i -o pmc --output-format csv -- \
    python3 scripts/run_workload.py $W 3 ${VARIANT:-} > $OUT/pmcsq_${TAG}_$i.log 2>&1; rc=$?
  tail -1 $OUT/pmcsq_${TAG}_$i.log; fatal $rc "pmc pass $i"
done
python3 - <<'PY'
import csv, glob, collections, os
W = os.environ["TAG"]
for path in sorted(glob.glob(f"gpurun_out/pmcsq_{W}_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "").split("(icrc::BatchParams")[0].split("(BatchParams")[0][:72]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        if "icrc" in k:
            print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
echo "== done"
