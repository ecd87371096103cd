#!/bin/bash
# scripts/gpu_r05_ringshape.sh — the submission ring's GPU tests, then the native message probe
# (scripts/msg_probe: configs[0]'s 64 x 4156-B message, compute + verify per message) on the launch
# path and on ring shapes ICRC_RING_SLOTS x ICRC_RING_WGS, 1 / 3 / 4 threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05b}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; *) echo "$2 exited $1"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 150 --timeout-method thread > $OUT/ring_tests.log 2>&1
rc=$?; tail -3 $OUT/ring_tests.log; fatal $rc ring-tests
MSG_PROBE_PATH=launch timeout -k 10 180 ./scripts/_build/msg_probe 1000 1 3 > $OUT/msg_launch.jsonl 2>&1; rc=$?; cat $OUT/msg_launch.jsonl; fatal $rc launch
for SH in ${SHAPES:-4x8 4x4 4x2 4x1 8x2}; do
  S=${SH%x*}; W=${SH#*x}
  echo "== ring $SH"
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W timeout -k 10 180 ./scripts/_build/msg_probe 1000 > $OUT/msg_ring_$SH.jsonl 2>&1; rc=$?; cat $OUT/msg_ring_$SH.jsonl; fatal $rc ring-$SH
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W timeout -k 10 180 ./scripts/_build/msg_probe 1000 1 3 4 > $OUT/msg_ring_thr_$SH.jsonl 2>&1; rc=$?; cat $OUT/msg_ring_thr_$SH.jsonl; fatal $rc ring-thr-$SH
done
echo "== done"
