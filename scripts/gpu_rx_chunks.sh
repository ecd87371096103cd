#!/bin/bash
# scripts/probe_rx_chunks.py under a kernel trace: per chunking, the summed durations of the verify
# pass (hybrid kernel) and of the descriptor pass.  Output: gpurun_out/rx_chunks/, rx_chunks.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/rx_chunks
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/rx_chunks -o run --output-format csv -- \
  python3 scripts/probe_rx_chunks.py 10 > $OUT/rx_chunks.jsonl 2> $OUT/rx_chunks.err
rc=$?; cat $OUT/rx_chunks.jsonl; tail -2 $OUT/rx_chunks.err
case $rc in 0) ;; *) echo "FATAL $rc"; exit $rc;; esac
python3 - <<'PY'
import csv, glob
rows = []
for path in glob.glob("gpurun_out/rx_chunks/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(path)))
rows = [r for r in rows if "hybrid" in r["Kernel_Name"] or "rx_desc" in r["Kernel_Name"] or "icrc_batch" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the probe's call sequence: for chunks in (1, 4, 8, 16, 1): (1 warm-up + 10 timed) x chunks rx_parse calls
seq, i = [], 0
for chunks in (1, 4, 8, 16, 1):
    n = 11 * chunks * 2
    seq.append((chunks, rows[i:i + n])); i += n
for chunks, rs in seq:
    ver = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs if "rx_desc" not in r["Kernel_Name"]]
    des = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs if "rx_desc" in r["Kernel_Name"]]
    print({"chunks": chunks, "verify_ms_per_batch": round(sum(ver) / 11 / 1e6, 4), "desc_ms_per_batch": round(sum(des) / 11 / 1e6, 4),
           "kernels": len(rs)})
PY
echo "== done"
