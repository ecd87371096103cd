#!/bin/bash
# scripts/gpu_r05_send.sh — the packetizer at wire slot strides 4156 / 4224 / 8192,
# then one PMC pass per stride with the write-request counters (TCC_EA0_WRREQ, _WRREQ_64B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05s}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; *) echo "$2 exited $1"; exit "$1";; esac; }
timeout -k 10 300 python3 scripts/probe_send.py 3 --strides 4156,4224,8192 > $OUT/probe_send_strides.jsonl 2> $OUT/probe_send.err
rc=$?; cat $OUT/probe_send_strides.jsonl; fatal $rc probe-send
for ST in 4156 4224 8192; do
  rm -rf $OUT/pmc_send_$ST
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B -d $OUT/pmc_send_$ST -o pmc --output-format csv -- \
    python3 scripts/probe_send.py 1 --strides $ST > $OUT/pmc_send_$ST.log 2>&1; rc=$?; tail -1 $OUT/pmc_send_$ST.log; fatal $rc pmc-$ST
done
python3 - <<'PY' | tee $OUT/pmc_send_summary.txt
import csv, glob, collections
for st in (4156, 4224, 8192):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for path in glob.glob(f"gpurun_out/${TAG:-r05s}/pmc_send_{st}/**/*counter_collection.csv".replace("${TAG:-r05s}", __import__("os").environ.get("TAG", "r05s")), recursive=True):
        for r in csv.DictReader(open(path)):
            if "packetize" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(st, {c: round(sum(v.values()) / max(1, len(v))) for c, v in acc.items()}, "dispatches", {c: len(v) for c, v in acc.items()})
PY
echo "== done"
