#!/bin/bash
# scripts/gpu_check.sh — one gpurun call: GPU tests, smoke, bench, rocprof kernel stats, and
# (PMC=1) the FETCH_SIZE / WRITE_SIZE passes for roofline.traffic.
# Every GPU step has its own time limit; a crash/timeout (124/134/137/139) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit status, $2 = step name
  case "$1" in
    124|134|137|139) echo "FATAL: $2 exited $1 — stopping"; exit "$1";;
  esac
}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== tests"
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --maxfail=5 --timeout 300 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1; rc=$?
  tail -5 $OUT/gpu_tests.log; stop_if_fatal $rc tests
  echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  tail -3 $OUT/smoke.log; stop_if_fatal $rc smoke
fi
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_if_fatal $rc bench
if [ "${PROFILE:-1}" = 1 ]; then
  echo "== rocprofv3"
  rm -rf $OUT/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu ${PROFILE_ARGS:-} > $OUT/prof.log 2>&1; rc=$?
  tail -3 $OUT/prof.log; stop_if_fatal $rc rocprof
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
fi
if [ "${PMC:-0}" = 1 ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C"
    rm -rf $OUT/pmc_bench_$C
    timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc_bench_$C -o pmc --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmc_bench_$C.log 2>&1; rc=$?
    tail -1 $OUT/pmc_bench_$C.log; stop_if_fatal $rc "pmc bench $C"
    if [ -x scripts/_build/membench ]; then
      rm -rf $OUT/pmc_mem_$C
      timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc_mem_$C -o pmc --output-format csv -- \
        ./scripts/_build/membench > $OUT/pmc_mem_$C.log 2>&1; rc=$?
      tail -1 $OUT/pmc_mem_$C.log; stop_if_fatal $rc "pmc membench $C"
    fi
  done
  python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.json; cat $OUT/pmc_summary.json
fi
echo "== done"
