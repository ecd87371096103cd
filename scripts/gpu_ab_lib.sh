#!/bin/bash
# A/B of two builds of the library on one box: alternating processes of scripts/ab_variants.py,
# the B build selected with ICRC_AMD_LIB (default: open-rdma-driver_amd/_build_ab/libicrc_amd_old.so).
# VARIANTS (default -1), JOBS (ab_variants.py), REPS (default 3).  Output: gpurun_out/ab_lib.jsonl, one line per
# (build, workload, variant) per repetition.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
B=${B_LIB:-open-rdma-driver_amd/_build_ab/libicrc_amd_old.so}
: > $OUT/ab_lib.jsonl
for i in $(seq ${REPS:-3}); do
  for build in new old; do
    if [ $build = old ]; then export ICRC_AMD_LIB=$PWD/$B; else unset ICRC_AMD_LIB; fi
    ROUNDS=${ROUNDS:-3} timeout -k 10 300 python3 scripts/ab_variants.py ${VARIANTS:--1} > $OUT/ab_one.jsonl 2> $OUT/ab_one.err; rc=$?
    case $rc in 0) ;; *) echo "FATAL: ab_variants ($build) exited $rc"; tail -5 $OUT/ab_one.err; exit $rc;; esac
    sed "s/^{/{\"build\": \"$build\", \"rep\": $i, /" $OUT/ab_one.jsonl >> $OUT/ab_lib.jsonl
  done
done
cat $OUT/ab_lib.jsonl
