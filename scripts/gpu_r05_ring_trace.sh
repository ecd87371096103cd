#!/bin/bash
# scripts/gpu_r05_ring_trace.sh — a ring job's phases on the GPU clock (A/B library, ICRC_RING_TRACE:
# cmd seen -> job decoded -> results complete -> done stored, and done -> next cmd seen), from
# scripts/msg_probe_ab at 1 and 3 threads (configs[0]'s 64 x 4156-B message) and on one packet.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05g}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "$2 exited $1"; exit "$1";; esac; }
cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1 || true
for T in 1 3; do
  echo "== threads $T"
  ICRC_RING_TRACE=1 ICRC_RING_AB=${AB:-0} timeout -k 10 120 ./scripts/_build/msg_probe_ab 1000 $T > $OUT/trace_t$T.jsonl 2>&1; rc=$?; cat $OUT/trace_t$T.jsonl; fatal $rc trace-$T
done
echo "== latency cases"
ICRC_RING_TRACE=1 ICRC_RING_AB=${AB:-0} timeout -k 10 120 ./scripts/_build/msg_probe_ab 1000 > $OUT/trace_lat.jsonl 2>&1; rc=$?; cat $OUT/trace_lat.jsonl; fatal $rc trace-lat
echo "== done"
