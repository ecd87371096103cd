#!/bin/bash
# A/B of two builds of the product library on one box: the python command CMD (a script under
# scripts/ printing JSON lines) run alternately with this tree's build ("new") and B_LIB ("old",
# default open-rdma-driver_amd/_build_ab/libicrc_amd_old.so) selected by ICRC_AMD_LIB, REPS times.
# Output: gpurun_out/ab_cmd.jsonl, each line tagged with build and rep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
B=${B_LIB:-open-rdma-driver_amd/_build_ab/libicrc_amd_old.so}
: > $OUT/ab_cmd.jsonl
for i in $(seq ${REPS:-3}); do
  for build in new old; do
    if [ $build = old ]; then export ICRC_AMD_LIB=$PWD/$B; else unset ICRC_AMD_LIB; fi
    timeout -k 10 300 python3 $CMD > $OUT/ab_cmd_one.jsonl 2> $OUT/ab_cmd_one.err; rc=$?
    case $rc in 0) ;; *) echo "FATAL: $CMD ($build) exited $rc"; tail -5 $OUT/ab_cmd_one.err; exit $rc;; esac
    sed "s/^{/{\"build\": \"$build\", \"rep\": $i, /" $OUT/ab_cmd_one.jsonl >> $OUT/ab_cmd.jsonl
  done
done
cat $OUT/ab_cmd.jsonl
