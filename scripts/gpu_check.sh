#!/bin/bash
# scripts/gpu_check.sh — one gpurun call: GPU tests, smoke, bench, rocprof kernel stats.
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
echo "== tests"; timeout -k 10 1200 python -m pytest tests -q -m gpu -x > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log; stop_if_fatal $rc tests
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -3 $OUT/smoke.log; stop_if_fatal $rc smoke
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_if_fatal $rc bench
if [ "${PROFILE:-1}" = 1 ]; then
  echo "== rocprofv3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof.log 2>&1; rc=$?
  tail -3 $OUT/prof.log; stop_if_fatal $rc rocprof
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
echo "== done"
