#!/bin/bash
# Every GPU test, smoke, then a same-box A/B of the product library against OLD (B_LIB) on C1,
# C1 verify, C2 and 316-byte packets (scripts/gpu_ab_lib.sh), then bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/skew_tests.log 2>&1; rc=$?; tail -2 gpurun_out/skew_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -3 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
B_LIB=${B_LIB:-open-rdma-driver_amd/_build_ab/old/libicrc_amd.so} VARIANTS=-1 JOBS=${JOBS:-C1,C1v,C2,S316} REPS=${REPS:-3} \
  bash scripts/gpu_ab_lib.sh > gpurun_out/skew_ab_lib.log 2>&1 || { tail -5 gpurun_out/skew_ab_lib.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cut -c1-200 gpurun_out/bench.json; exit $rc
