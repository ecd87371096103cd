#!/bin/bash
# scripts/gpu_r05_ringshape3.sh — the service kernel's workgroup size (ICRC_RING_THREADS): one
# workgroup per CU either way (the table image), so 256-thread workgroups spread a job's loads over
# more CUs (scripts/hostreadbench.hip: one CU pulls host memory at ~25 GB/s, four at ~56).  The ring's
# GPU tests under each shape, then scripts/msg_probe at 1 / 3 / 4 threads, CONF "SLOTSxWGSxTHREADS",
# two alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05i}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "$2 exited $1"; exit "$1";; esac; }
for C in ${TESTCONFS:-4x4x256 4x2x1024}; do
  S=${C%%x*}; R=${C#*x}; W=${R%%x*}; T=${R#*x}
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W ICRC_RING_THREADS=$T timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py -x -q --timeout 150 --timeout-method thread > $OUT/ring_tests_$C.log 2>&1
  rc=$?; echo "tests $C: $(tail -1 $OUT/ring_tests_$C.log)"; fatal $rc ring-tests-$C
done
for R in 1 2; do
for C in ${CONFS:-4x2x1024 4x4x256 4x8x256 4x4x512 4x2x256}; do
  S=${C%%x*}; RR=${C#*x}; W=${RR%%x*}; T=${RR#*x}
  echo "== ring $C round $R"
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W ICRC_RING_THREADS=$T timeout -k 10 180 ./scripts/_build/msg_probe 1000 1 3 4 > $OUT/msg_ring_${C}_$R.jsonl 2>&1; rc=$?
  grep '"pinned, ring"' $OUT/msg_ring_${C}_$R.jsonl; fatal $rc ring-$C
  ICRC_RING_SLOTS=$S ICRC_RING_WGS=$W ICRC_RING_THREADS=$T timeout -k 10 180 ./scripts/_build/msg_probe 1000 > $OUT/msg_lat_${C}_$R.jsonl 2>&1; rc=$?
  grep 'pinned' $OUT/msg_lat_${C}_$R.jsonl; fatal $rc lat-$C
done
done
echo "== done"
