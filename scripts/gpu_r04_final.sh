#!/bin/bash
# scripts/gpu_r04_final.sh — the round's record on one box: every GPU test, smoke, the plain bench,
# rocprof kernel stats of the plain bench, the FETCH_SIZE / WRITE_SIZE passes (roofline.traffic),
# then bench --extra (every other config and section-8f row, incl. the native-thread message rate).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMC=1 bash scripts/gpu_check.sh || exit $?
timeout -k 10 900 python3 bench.py --extra --steps 20 --warmup 5 > gpurun_out/bench_extra.json 2> gpurun_out/bench_extra.err; rc=$?
tail -2 gpurun_out/bench_extra.err; case $rc in 0) ;; *) echo "bench --extra rc=$rc"; exit $rc;; esac
echo "== final done"
