#!/bin/bash
# scripts/gpu_r06_teardown.sh — one gpurun call for VERDICT r05 item 1 (the exit-time SIGSEGV under
# rocprofv3 after Python threads used the submission ring): the ring GPU tests (the new exit test
# included), then ONE profiled run of the leg that crashed (bench.py --only msg) with the address map
# dumped at the end of Python's exit path, then (only if that exits 0) the profiled --extra run whose
# kernel stats the round-5 records lacked.  Every GPU step has its own limit; a crash stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06_teardown
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {
  case "$1" in
    0) ;;
    *) echo "STOP: $2 exited $1"; exit "$1";;
  esac
}
echo "== ring tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_parity.py::test_rx_parse_mixed_mtu_stream_full -x -v --timeout 120 --timeout-method thread \
  > $OUT/ring_tests.log 2>&1; rc=$?
tail -15 $OUT/ring_tests.log; stop_if_fatal $rc ring_tests
echo "== rocprofv3 --only msg"
BENCH_DUMP_MAPS=$PWD/$OUT/msg_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_msg -o run \
  --output-format csv -- python3 bench.py --only msg --no-cpu --steps 5 --warmup 2 > $OUT/msg.log 2>&1; rc=$?
tail -25 $OUT/msg.log; stop_if_fatal $rc prof_msg
echo "== rocprofv3 --extra"
BENCH_DUMP_MAPS=$PWD/$OUT/extra_maps.txt timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_extra -o run \
  --output-format csv -- python3 bench.py --extra --no-cpu > $OUT/extra.json 2> $OUT/extra.err; rc=$?
tail -5 $OUT/extra.err; stop_if_fatal $rc prof_extra
find $OUT/prof_extra -name "*kernel_stats.csv" -exec cat {} \;
echo "== ring cost to device batches"
for m in "product" "ab 0" "ab 1"; do
  set -- $m
  ICRC_AB_RING_AWARE=${2:-1} timeout -k 10 120 python3 scripts/probe_ring_c1.py $1 >> $OUT/ring_c1.jsonl 2>> $OUT/ring_c1.err; rc=$?
  stop_if_fatal $rc "ring_c1 $m"
done
cat $OUT/ring_c1.jsonl
echo "== c3 decomposition (rocprof kernel trace)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- \
  python3 scripts/probe_c3_decomp.py > $OUT/c3_decomp.jsonl 2> $OUT/c3_decomp.err; rc=$?
tail -3 $OUT/c3_decomp.err; stop_if_fatal $rc c3_decomp
find $OUT/prof_c3 -name "*kernel_stats.csv" -exec cat {} \;
echo "== done"
