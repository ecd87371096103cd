#!/bin/bash
# LDS / issue counters over one workload (scripts/run_workload.py), one rocprofv3 --pmc run per
# pass: bank conflicts, LDS and VALU activity, GPU clock (GRBM_GUI_ACTIVE) — is the short-packet
# kernel LDS-, VALU- or latency-bound?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
W=${WORKLOAD:-s316}; TAG=${W}_${VARIANT:-dflt}; export TAG
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
i=0
for SET in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  rm -rf $OUT/pmclds_${TAG}_$i
  timeout -s KILL 120 rocprofv3 --pmc $SET -d $OUT/pmclds_${TAG}_$i -o pmc --output-format csv -- \
    python3 scripts/run_workload.py $W 3 ${VARIANT:-} > $OUT/pmclds_${TAG}_$i.log 2>&1; rc=$?
  tail -1 $OUT/pmclds_${TAG}_$i.log; fatal $rc "pmc pass $i"
done
python3 - <<'PY'
import csv, glob, collections, os
W = os.environ["TAG"]
for path in sorted(glob.glob(f"gpurun_out/pmclds_{W}_*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "").split("(icrc::BatchParams")[0].split("(BatchParams")[0][:72]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        if any(t in k for t in ("icrc_oct", "icrc_batch", "icrc_hybrid", "icrc_long")):
            print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
PY
echo "== done"
