#!/bin/bash
# Oct work-skew sweep (scripts/probe_skew.py, A/B library) + the per-slot end times of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-5} JOBS=${JOBS:-C2,S316,C2k,C2m} timeout -k 10 600 python scripts/probe_skew.py ${SKEWS:-0/0,12333/0,45/0,60/0,75/0,90/0} \
  > gpurun_out/skew_sweep.jsonl 2> gpurun_out/skew_sweep.err; rc=$?
cut -c1-100 gpurun_out/skew_sweep.jsonl; tail -2 gpurun_out/skew_sweep.err; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_oct_balance.py > gpurun_out/oct_balance_skew.jsonl 2> gpurun_out/oct_balance_skew.err; rc=$?
cut -c1-300 gpurun_out/oct_balance_skew.jsonl; exit $rc
