#!/bin/bash
# scripts/gpu_r05_ringshape2.sh — ring shape / lifetime choice: the ring's GPU tests, then
# scripts/msg_probe (configs[0]'s 64 x 4156-B message, compute + verify) at 1 / 3 / 4 threads for each
# CONF "SLOTSxWGS:LIFE_US", twice in alternation (box noise), and the launch path once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "$2 exited $1"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 150 --timeout-method thread > $OUT/ring_tests.log 2>&1
rc=$?; tail -3 $OUT/ring_tests.log; fatal $rc ring-tests
MSG_PROBE_PATH=launch timeout -k 10 180 ./scripts/_build/msg_probe 1000 1 3 > $OUT/msg_launch.jsonl 2>&1; rc=$?; cat $OUT/msg_launch.jsonl; fatal $rc launch
for R in 1 2; do
for C in ${CONFS:-4x2:1000 4x4:1000 4x2:3000 4x4:3000}; do
  SH=${C%:*}; LIFE=${C#*:}; S=${SH%x*}; W=${SH#*x}
  echo "== ring $C round $R"
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W ICRC_RING_LIFE_US=$LIFE timeout -k 10 180 ./scripts/_build/msg_probe 1000 1 3 4 > $OUT/msg_ring_${SH}_${LIFE}_$R.jsonl 2>&1; rc=$?; cat $OUT/msg_ring_${SH}_${LIFE}_$R.jsonl; fatal $rc ring-$C
done
done
echo "== done"
