#!/bin/bash
# scripts/gpu_r05_ring_ab.sh — where a ring job's fixed time goes: the A/B library's diagnostic
# cuts of the ring kernel (ICRC_RING_AB: 1 no acquire, 2 release fence added, 4 no sleep between polls,
# 8 no compute — results wrong for 8, rate only) under scripts/msg_probe_ab, 1 thread and 3 threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r05e}; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "$2 exited $1"; exit "$1";; esac; }
for AB in ${ABS:-0 1 2 4 8 3 15 0}; do
  echo "== ab $AB"
  ICRC_RING_SLOTS=${S:-4} ICRC_RING_WGS=${W:-2} ICRC_RING_AB=$AB timeout -k 10 120 ./scripts/_build/msg_probe_ab 1000 > $OUT/ab_${AB}_lat.jsonl 2>&1; rc=$?; cat $OUT/ab_${AB}_lat.jsonl; fatal $rc ab-$AB
  ICRC_RING_SLOTS=${S:-4} ICRC_RING_WGS=${W:-2} ICRC_RING_AB=$AB timeout -k 10 120 ./scripts/_build/msg_probe_ab 1000 3 > $OUT/ab_${AB}_thr.jsonl 2>&1; rc=$?; cat $OUT/ab_${AB}_thr.jsonl; fatal $rc ab-thr-$AB
done
echo "== done"
