#!/bin/bash
# tests + variant A/B (one process) + optional rocprof of the A/B; stops on fatal exit codes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
if [ "${TESTS:-1}" = 1 ]; then
  echo "== tests"; timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:--x} > $OUT/gpu_tests.log 2>&1; rc=$?
  tail -4 $OUT/gpu_tests.log; fatal $rc tests
fi
echo "== ab"; timeout -k 10 400 python scripts/ab_variants.py ${VARIANTS:-16,13,0} > $OUT/ab.json 2> $OUT/ab.err; rc=$?
cat $OUT/ab.json; tail -3 $OUT/ab.err; fatal $rc ab
echo "== done"
