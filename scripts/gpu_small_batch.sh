#!/bin/bash
# Small batches (one WRITE message of 64 / 1024 / 4096 4-KiB packets, compute only): kernel
# durations on the GPU (rocprofv3 kernel trace) against the per-launch time the A/B script's
# events see for back-to-back launches — how much of a small batch is the kernel and how much the
# launch.  Output: gpurun_out/small_batch/ (kernel_stats.csv, kernel_trace.csv), small_batch.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/small_batch
JOBS=W64,W1024,C3c ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/small_batch -o run --output-format csv -- \
  python3 scripts/ab_variants.py -1 > $OUT/small_batch.jsonl 2> $OUT/small_batch.err
rc=$?; cat $OUT/small_batch.jsonl; tail -2 $OUT/small_batch.err
case $rc in 124|134|137|139) echo "FATAL $rc"; exit $rc;; esac
python3 - <<'PY'
import csv, glob, collections
for path in glob.glob("gpurun_out/small_batch/**/*kernel_trace.csv", recursive=True):
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if "icrc_batch_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        key = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        gap = (s - prev_end) if prev_end is not None else None
        by[key].append((e - s, gap))
        prev_end = e
    for k, v in by.items():
        d = sorted(x[0] for x in v); g = sorted(x[1] for x in v if x[1] is not None and x[1] < 100000)
        print("grid", k, "launches", len(v), "kernel ns median", d[len(d) // 2], "min", d[0],
              "gap to previous ns median", g[len(g) // 2] if g else None)
PY
echo "== done"
