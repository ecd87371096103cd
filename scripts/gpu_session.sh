#!/bin/bash
# scripts/gpu_session.sh — one gpurun call of ordered steps, each under its own time limit; a
# crash / timeout (124/134/137/139) stops the script.  STEPS (comma list) picks from:
#   tests   pytest -m gpu (all)          smoke   __graft_entry__.smoke()
#   bench   bench.py (default)           extra   bench.py --extra
#   probe   scripts/probe_packetize_alloc.py
#   prof    rocprofv3 --kernel-trace --stats of bench.py --no-cpu
# TESTS_K: a pytest -k expression for the tests step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {
  case "$1" in
    124|134|137|139) echo "FATAL: $2 exited $1 — stopping"; exit "$1";;
  esac
}
IFS=, read -ra S <<< "${STEPS:-tests,smoke,bench}"
for step in "${S[@]}"; do
  case $step in
    tests)
      echo "== tests"
      timeout -k 10 900 python -u -m pytest tests -q -m gpu ${TESTS_K:+-k "$TESTS_K"} --maxfail=5 --timeout 300 \
        --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
      tail -8 $OUT/gpu_tests.log; stop_if_fatal $rc tests;;
    smoke)
      echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      tail -3 $OUT/smoke.log; stop_if_fatal $rc smoke;;
    bench)
      echo "== bench"; timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_if_fatal $rc bench;;
    extra)
      echo "== bench --extra"; timeout -k 10 900 python bench.py --extra > $OUT/bench_extra.json 2> $OUT/bench_extra.err; rc=$?
      cat $OUT/bench_extra.json; tail -3 $OUT/bench_extra.err; stop_if_fatal $rc extra;;
    probe)
      echo "== probe packetize"; timeout -k 10 600 python scripts/probe_packetize_alloc.py > $OUT/probe_pk.jsonl 2> $OUT/probe_pk.err; rc=$?
      cat $OUT/probe_pk.jsonl; tail -3 $OUT/probe_pk.err; stop_if_fatal $rc probe;;
    prof)
      echo "== rocprofv3"; rm -rf $OUT/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --no-cpu > $OUT/prof.log 2>&1; rc=$?
      tail -3 $OUT/prof.log; stop_if_fatal $rc prof
      find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; ;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo "== done"
