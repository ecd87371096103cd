#!/bin/bash
# scripts/gpu_pmc.sh — HBM traffic counters for the ICRC kernel (roofline.traffic).
# Separate rocprofv3 passes for FETCH_SIZE and WRITE_SIZE (they do not fit one TCC pass),
# counters only (no sys/runtime trace).  The same passes over scripts/membench (known byte
# counts per pattern) calibrate FETCH_SIZE for these access widths on gfx950.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== bench $C"
  timeout -k 10 600 rocprofv3 --pmc $C -d $OUT/pmc_bench_$C -o pmc --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmc_bench_$C.log 2>&1; rc=$?
  tail -2 $OUT/pmc_bench_$C.log; fatal $rc "bench $C"
  echo "== membench $C"
  timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc_mem_$C -o pmc --output-format csv -- \
    ./scripts/membench > $OUT/pmc_mem_$C.log 2>&1; rc=$?
  tail -2 $OUT/pmc_mem_$C.log; fatal $rc "membench $C"
done
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json; cat $OUT/pmc_summary.json
echo "== done"
