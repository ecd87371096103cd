#!/bin/bash
# Instruction mix of the oct kernel and its ablations on 4 Mi strided 316-B packets (one set =
# one frame = 8 packets): SQ_INSTS_* per dispatch for variants 40 (full), 41 (loads only), 43
# (control + final products), 44 (control only).  One rocprofv3 --pmc pass per variant.
# Output: gpurun_out/pmc_oct_insts.txt (per dispatch, and per set = 4 Mi / 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
for V in ${VARIANTS:-40 41 43 44}; do
  rm -rf $OUT/pmcoi_$V
  timeout -s KILL 150 rocprofv3 --pmc $CTR -d $OUT/pmcoi_$V -o pmc --output-format csv -- \
    python3 scripts/run_workload.py ${WORKLOAD:-s316} 3 $V > $OUT/pmcoi_$V.log 2>&1
  rc=$?; tail -1 $OUT/pmcoi_$V.log
  case $rc in 0) ;; *) echo "FATAL pmc $V rc=$rc"; exit $rc;; esac
done
python3 - <<'PY' | tee $OUT/pmc_oct_insts.txt
import csv, glob, collections, os
sets = (4 << 20) / 8
for V in os.environ.get("VARIANTS", "40 41 43 44").split():
    acc = collections.defaultdict(float); disp = set()
    for path in glob.glob(f"gpurun_out/pmcoi_{V}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if "icrc_oct_kernel" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r.get("Dispatch_Id"))
    nd = max(1, len(disp))
    print("variant", V, "dispatches", nd, {k: round(v / nd / sets, 2) for k, v in sorted(acc.items())}, "(per set)")
PY
echo "== done"
