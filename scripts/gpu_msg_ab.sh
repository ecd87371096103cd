#!/bin/bash
# Per-message latency A/B of two library builds (scripts/_build/msg_probe, configs[0]'s shape):
# the new build (open-rdma-driver_amd/_build) and OLD_DIR's libicrc_amd.so (LD_LIBRARY_PATH wins
# over the probe's RUNPATH), alternating, REPS times.  Then the host-batch GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
OLD=${OLD_DIR:-open-rdma-driver_amd/_build_ab/old}
: > $OUT/msg_ab.jsonl
for i in $(seq ${REPS:-3}); do
  for build in new old; do
    if [ $build = old ]; then LP=$PWD/$OLD; else LP=; fi
    LD_LIBRARY_PATH=$LP timeout -k 10 120 scripts/_build/msg_probe ${CALLS:-2000} > $OUT/msg_one.jsonl 2> $OUT/msg_one.err; rc=$?
    case $rc in 0) ;; *) echo "FATAL: msg_probe ($build) exited $rc"; tail -5 $OUT/msg_one.err; exit $rc;; esac
    sed "s/^{/{\"build\": \"$build\", \"rep\": $i, /" $OUT/msg_one.jsonl >> $OUT/msg_ab.jsonl
  done
done
cat $OUT/msg_ab.jsonl
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "host or scalar or message or batch" > $OUT/msg_tests.log 2>&1; rc=$?
  tail -3 $OUT/msg_tests.log; exit $rc
fi
