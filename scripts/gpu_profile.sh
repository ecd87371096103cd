#!/bin/bash
# scripts/gpu_profile.sh — one gpurun call: rocprofv3 kernel statistics of bench.py --extra (every
# case's kernels), then FETCH_SIZE / WRITE_SIZE passes (separate runs, PMC only) over the C1 bench,
# the fused send packetizer and membench's calibration shapes; summary -> gpurun_out/pmc_summary.json.
# Every GPU step has its own time limit; a crash/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1 — stopping"; exit "$1";; esac; }
echo "== rocprofv3 --stats (bench --extra)"
rm -rf $OUT/prof_extra
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_extra -o run --output-format csv -- \
  python3 bench.py --extra --steps 10 --warmup 2 --no-cpu > $OUT/prof_extra.log 2>&1; rc=$?
tail -2 $OUT/prof_extra.log; stop_if_fatal $rc rocprof
find $OUT/prof_extra -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_extra.csv \;
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  rm -rf $OUT/pmc_bench_$C $OUT/pmc_packetize_$C $OUT/pmc_mem_$C
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_bench_$C -o pmc --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmc_bench_$C.log 2>&1; rc=$?
  tail -1 $OUT/pmc_bench_$C.log; stop_if_fatal $rc "pmc bench $C"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_packetize_$C -o pmc --output-format csv -- \
    python3 scripts/run_workload.py packetize 3 > $OUT/pmc_packetize_$C.log 2>&1; rc=$?
  tail -1 $OUT/pmc_packetize_$C.log; stop_if_fatal $rc "pmc packetize $C"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_mem_$C -o pmc --output-format csv -- \
    ./scripts/_build/membench > $OUT/pmc_mem_$C.log 2>&1; rc=$?
  tail -1 $OUT/pmc_mem_$C.log; stop_if_fatal $rc "pmc membench $C"
done
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json; tail -30 $OUT/pmc_summary.json
echo "== done"
