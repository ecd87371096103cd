#!/bin/bash
# Instruction-cache counters (SQC_ICACHE_*, SQ_IFETCH) next to the issue-wait counters for the
# default kernels of C1, C2, the 256-B class alone and 4 Mi strided 316-B packets: does the
# short-packet ring (tens of KiB of unrolled code; the hybrid launch carries the long-packet body
# as well) miss in the instruction cache two CUs share?  One rocprofv3 --pmc pass per workload.
# Output: gpurun_out/pmc_icache_summary.txt (per kernel, per dispatch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
CTR="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU"
for W in ${WORKLOADS:-c1 c2 c2s s316}; do
  rm -rf $OUT/pmcic_$W
  timeout -s KILL 150 rocprofv3 --pmc $CTR -d $OUT/pmcic_$W -o pmc --output-format csv -- \
    python3 scripts/run_workload.py $W 3 ${VARIANT:-} > $OUT/pmcic_$W.log 2>&1
  rc=$?; tail -1 $OUT/pmcic_$W.log; fatal $rc "pmc $W"
done
python3 - <<'PY' | tee $OUT/pmc_icache_summary.txt
import csv, glob, collections, os
for W in os.environ.get("WORKLOADS", "c1 c2 c2s s316").split():
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for path in glob.glob(f"gpurun_out/pmcic_{W}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("icrc::", "")
            k = k.split("(icrc::BatchParams")[0].split("(BatchParams")[0][:90]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r.get("Dispatch_Id"))
    for k, d in sorted(acc.items()):
        if "synth" in k:
            continue
        nd = max(1, len(disp[k]))
        v = {c: round(x / nd, 1) for c, x in sorted(d.items())}
        req = v.get("SQC_ICACHE_REQ", 0) or 1
        print(W, "|", k, "| dispatches", nd, "| miss/req %.4f" % (v.get("SQC_ICACHE_MISSES", 0) / req),
              "| wait_inst/wave_cycles %.3f" % (v.get("SQ_WAIT_INST_ANY", 0) / (v.get("SQ_WAVE_CYCLES", 0) or 1)), "|", v)
PY
echo "== done"
