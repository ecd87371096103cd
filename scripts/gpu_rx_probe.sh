#!/bin/bash
# Receive parse on 4 Mi x 316 B (scripts/run_workload.py rx316 / rx316r): kernel durations
# (rocprofv3 --kernel-trace --stats), then FETCH_SIZE / WRITE_SIZE per kernel (scripts/gpu_pmc_traffic.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
for W in ${WORKLOADS:-rx316 rx316r}; do
  rm -rf $OUT/rxprof_$W
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/rxprof_$W -o run --output-format csv -- \
    python3 scripts/run_workload.py $W 10 ${VARIANT:-} > $OUT/rxprof_$W.log 2>&1; rc=$?
  tail -1 $OUT/rxprof_$W.log; fatal $rc "stats $W"
  find $OUT/rxprof_$W -name "*kernel_stats.csv" -exec cp {} $OUT/rxprof_${W}_stats.csv \;
  cut -c1-160 $OUT/rxprof_${W}_stats.csv | head -8
  WORKLOAD=$W bash scripts/gpu_pmc_traffic.sh || exit $?
done
echo "== done"
