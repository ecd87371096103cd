#!/bin/bash
# scripts/gpu_r05_ring.sh — round 5, first box: the submission-ring GPU tests first (new code), then
# every GPU test, smoke, the native message probe on both host paths, and the default bench line
# (headline + configs[2] / configs[3]).  Each GPU step has its own time limit; a crash / timeout ends
# the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05a}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; *) echo "$2 exited $1";; esac; }
echo "== ring tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -x -v --timeout 150 --timeout-method thread > $OUT/ring_tests.log 2>&1
rc=$?; tail -12 $OUT/ring_tests.log; fatal $rc ring-tests; [ $rc = 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; fatal $rc gpu-tests; [ $rc = 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; fatal $rc smoke; [ $rc = 0 ] || exit $rc
echo "== msg_probe"
for P in ring launch; do
  MSG_PROBE_PATH=$P timeout -k 10 180 ./scripts/_build/msg_probe 2000 > $OUT/msg_$P.jsonl 2>&1; rc=$?; cat $OUT/msg_$P.jsonl; fatal $rc msg-$P; [ $rc = 0 ] || exit $rc
  MSG_PROBE_PATH=$P timeout -k 10 180 ./scripts/_build/msg_probe 2000 1 3 4 > $OUT/msg_thr_$P.jsonl 2>&1; rc=$?; cat $OUT/msg_thr_$P.jsonl; fatal $rc msg-thr-$P; [ $rc = 0 ] || exit $rc
done
echo "== bench"
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cat $OUT/bench.json; tail -3 $OUT/bench.err; fatal $rc bench
echo "== done"
