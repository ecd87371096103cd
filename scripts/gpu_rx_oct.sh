#!/bin/bash
# The one-pass strided receive (icrc_oct_rx_kernel): receive parity tests, bench.py --only rx, and
# kernel statistics of run_workload.py rx316 with the one pass (default) and the two passes
# (ICRC_AB_RX_OCT=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "rx_parse or receive" > $OUT/rxoct_tests.log 2>&1; rc=$?
tail -3 $OUT/rxoct_tests.log; fatal $rc tests
timeout -k 10 300 python3 bench.py --only rx --steps 20 --warmup 5 --no-cpu > $OUT/rxoct_bench.log 2>&1; rc=$?
tail -1 $OUT/rxoct_bench.log | cut -c1-600; fatal $rc bench
for AB in 1 0; do
  rm -rf $OUT/rxoct_prof_$AB
  ICRC_AB_RX_OCT=$AB timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/rxoct_prof_$AB -o run --output-format csv -- \
    python3 scripts/run_workload.py rx316 20 > $OUT/rxoct_prof_$AB.log 2>&1; rc=$?
  tail -1 $OUT/rxoct_prof_$AB.log; fatal $rc "prof $AB"
  find $OUT/rxoct_prof_$AB -name "*kernel_stats.csv" -exec cp {} $OUT/rxoct_stats_$AB.csv \;
  echo "== ICRC_AB_RX_OCT=$AB"; cut -d, -f1-4 $OUT/rxoct_stats_$AB.csv | cut -c1-150 | head -6
done
echo "== done"
