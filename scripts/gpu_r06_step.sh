#!/bin/bash
# scripts/gpu_r06_step.sh — one gpurun call of round 6's build -> measure loop.
#   TESTS   pytest selection run first (-m gpu), e.g. "tests/test_gpu_parity.py -k rx_parse"; empty = none
#   BENCH   bench.py arguments of a plain run after the tests (empty = none), e.g. "--only rx --no-cpu"
#   PROBES  ';'-separated commands run last, each under its own 300 s limit (measurement scripts)
#   TAG     output directory under gpurun_out/
# Every GPU step has its own limit; the first failing step ends the call (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_step}
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {
  case "$1" in
    0) ;;
    *) echo "STOP: $2 exited $1"; exit "$1";;
  esac
}
if [ -n "${TESTS:-}" ]; then
  echo "== tests: $TESTS"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/tests.log" 2>&1; rc=$?
  tail -15 "$OUT/tests.log"; stop_if_fatal $rc tests
fi
if [ -n "${BENCH:-}" ]; then
  echo "== bench $BENCH"
  timeout -k 10 600 python bench.py $BENCH > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
  cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; stop_if_fatal $rc bench
fi
if [ -n "${PROBES:-}" ]; then
  IFS=';' read -ra CMDS <<< "$PROBES"
  k=0
  for c in "${CMDS[@]}"; do
    k=$((k + 1))
    echo "== probe $k: $c"
    timeout -k 10 300 bash -c "$c" > "$OUT/probe_$k.out" 2> "$OUT/probe_$k.err"; rc=$?
    tail -40 "$OUT/probe_$k.out"; tail -3 "$OUT/probe_$k.err"; stop_if_fatal $rc "probe $k"
  done
fi
echo "== done"
