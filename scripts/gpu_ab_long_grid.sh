#!/bin/bash
# C2 with 1x / 2x / 4x long-packet workgroups per oct workgroup in the hybrid launch (A/B build,
# ICRC_AB_LONG_GRID), alternating processes.  (A second knob that put the long-packet workgroups
# first measured within noise, profiles/r03_ab_long_first.jsonl, and was removed again.)  Output: gpurun_out/ab_long_grid.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/ab_long_grid.jsonl
export ICRC_AMD_LIB=$PWD/open-rdma-driver_amd/_build/libicrc_amd_ab.so
for rep in 1 2 3; do
  for m in ${MULTS:-1 2 4}; do
    ICRC_AB_LONG_GRID=$m JOBS=${JOBS:-C2,C2k} ROUNDS=3 timeout -k 10 200 python3 scripts/ab_variants.py -1 > $OUT/ab_one.jsonl 2> $OUT/ab_one.err; rc=$?
    case $rc in 0) ;; *) echo "FATAL rc=$rc"; tail -3 $OUT/ab_one.err; exit $rc;; esac
    sed "s/^{/{\"long_grid_mult\": $m, \"rep\": $rep, /" $OUT/ab_one.jsonl >> $OUT/ab_long_grid.jsonl
  done
done
cat $OUT/ab_long_grid.jsonl
