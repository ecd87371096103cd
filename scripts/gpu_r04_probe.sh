#!/bin/bash
# scripts/gpu_r04_probe.sh — one gpurun call: the submitter's message rate from 1-4 threads
# (scripts/_build/msg_probe, C++), then the C2 mix decomposition (scripts/ab_variants.py, default
# dispatch).  Every GPU step has its own time limit; a crash / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
stop_if_fatal() { case "$1" in 0) ;; *) echo "FATAL: $2 exited $1 — stopping"; exit "$1";; esac; }
if [ -n "${TESTK:-}" ]; then  # a subset of the GPU tests first (pytest -k expression)
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -k "$TESTK" --timeout 120 --timeout-method thread \
    > $OUT/gpu_tests_sub.log 2>&1; rc=$?
  tail -3 $OUT/gpu_tests_sub.log; stop_if_fatal $rc tests
fi
if [ "${PLACE:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u scripts/probe_packetize_place.py > $OUT/pk_place.jsonl 2> $OUT/pk_place.err; rc=$?
  cat $OUT/pk_place.jsonl; tail -3 $OUT/pk_place.err; stop_if_fatal $rc probe_packetize_place
fi
if [ "${SPLIT:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u scripts/probe_split.py > $OUT/c2_split.jsonl 2> $OUT/c2_split.err; rc=$?
  cat $OUT/c2_split.jsonl; tail -3 $OUT/c2_split.err; stop_if_fatal $rc probe_split
fi
if [ -n "${AB_ENV:-}" ]; then
  timeout -k 10 600 python3 -u scripts/probe_env_ab.py > $OUT/env_ab.jsonl 2> $OUT/env_ab.err; rc=$?
  cat $OUT/env_ab.jsonl; tail -3 $OUT/env_ab.err; stop_if_fatal $rc probe_env_ab
fi
if [ -n "${SPREAD_VALUES:-}" ]; then  # msg_probe on the A/B library, one run per ICRC_AB_SPREAD value
  mkdir -p /tmp/icrc_ablib && ln -sf "$PWD/open-rdma-driver_amd/_build/libicrc_amd_ab.so" /tmp/icrc_ablib/libicrc_amd.so
  for v in $SPREAD_VALUES; do
    ICRC_AB_SPREAD=$v LD_LIBRARY_PATH=/tmp/icrc_ablib timeout -k 10 240 scripts/_build/msg_probe ${CALLS:-2000} 1 3 4 \
      > $OUT/msg_spread_$v.jsonl 2> $OUT/msg_spread_$v.err; rc=$?
    sed "s/^{/{\"spread_per_wg\": $v, /" $OUT/msg_spread_$v.jsonl; stop_if_fatal $rc msg_probe_spread
  done
fi
if [ "${PRESORT:-0}" = 1 ]; then
  timeout -k 10 600 python3 -u scripts/probe_presort.py > $OUT/presort.jsonl 2> $OUT/presort.err; rc=$?
  cat $OUT/presort.jsonl; tail -3 $OUT/presort.err; stop_if_fatal $rc probe_presort
fi
if [ "${MSGAB:-0}" = 1 ]; then  # the round-3 library (one launch in flight) vs this build, alternating
  # (recorded in profiles/r04_msg_submitter_ab.jsonl; _build/old_r03 is gpurun-ignored since: un-ignore to rerun)
  for r in 1 2; do
    for b in old_r03 new; do
      d=open-rdma-driver_amd/_build; [ $b = old_r03 ] && d=open-rdma-driver_amd/_build/old_r03
      LD_LIBRARY_PATH=$d timeout -k 10 240 scripts/_build/msg_probe ${CALLS:-2000} 1 3 > $OUT/msgab_$b.jsonl 2> $OUT/msgab_$b.err; rc=$?
      sed "s/^{/{\"build\": \"$b\", \"round\": $r, /" $OUT/msgab_$b.jsonl; stop_if_fatal $rc msg_probe_ab
    done
  done
fi
if [ "${MSG:-1}" = 1 ]; then
  LD_LIBRARY_PATH=open-rdma-driver_amd/_build timeout -k 10 240 scripts/_build/msg_probe ${CALLS:-2000} 1 2 3 4 \
    > $OUT/msg_threads.jsonl 2> $OUT/msg_threads.err; rc=$?
  cat $OUT/msg_threads.jsonl; stop_if_fatal $rc msg_probe
fi
if [ "${DECOMP:-1}" = 1 ]; then
  JOBS=${DJOBS:-C2,C2short,C2long,C2nr,C2s,C2snr,C2k,C2m,S316} ROUNDS=${ROUNDS:-3} timeout -k 10 600 \
    python3 -u scripts/ab_variants.py ${VARIANTS:--1} > $OUT/c2_decomp.jsonl 2> $OUT/c2_decomp.err; rc=$?
  cat $OUT/c2_decomp.jsonl; tail -3 $OUT/c2_decomp.err; stop_if_fatal $rc ab_variants
fi
echo "== done"
