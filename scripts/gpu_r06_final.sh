#!/bin/bash
# scripts/gpu_r06_final.sh — round 6's record run, one gpurun call: every GPU test + smoke, the
# default bench line, the profiled --extra run (rocprofv3 kernel trace), the FETCH_SIZE / WRITE_SIZE
# passes behind roofline.traffic and configs.c2.traffic_ratio (with membench's calibration), and the
# packetizer's request counters against the copy shapes.  Output: gpurun_out/r06_final/.
# Every GPU step has its own limit; the first failing step ends the call (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06_final}
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {
  case "$1" in
    0) ;;
    *) echo "STOP: $2 exited $1"; exit "$1";;
  esac
}
if [ "${TESTS:-1}" = 1 ]; then
  echo "== gpu tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
  tail -4 "$OUT/gpu_tests.log"; stop_if_fatal $rc tests
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  tail -2 "$OUT/smoke.log"; stop_if_fatal $rc smoke
fi
if [ "${BENCH:-1}" = 1 ]; then
  echo "== bench (default line)"
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
  cut -c1-400 "$OUT/bench.json"; tail -2 "$OUT/bench.err"; stop_if_fatal $rc bench
  echo "== rocprofv3 kernel trace of bench.py --extra"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_extra" -o run --output-format csv -- \
    python3 bench.py --extra --no-cpu > "$OUT/bench_extra.json" 2> "$OUT/bench_extra.err"; rc=$?
  tail -2 "$OUT/bench_extra.err"; stop_if_fatal $rc prof_extra
fi
if [ "${PMC:-1}" = 1 ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C"
    timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/pmc_bench_$C" -o pmc --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu > "$OUT/pmc_bench_$C.log" 2>&1; rc=$?
    tail -1 "$OUT/pmc_bench_$C.log"; stop_if_fatal $rc "pmc bench $C"
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_mem_$C" -o pmc --output-format csv -- \
      ./scripts/_build/membench > "$OUT/pmc_mem_$C.log" 2>&1; rc=$?
    tail -1 "$OUT/pmc_mem_$C.log"; stop_if_fatal $rc "pmc membench $C"
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_packetize_$C" -o pmc --output-format csv -- \
      python3 scripts/run_workload.py packetize 3 > "$OUT/pmc_packetize_$C.log" 2>&1; rc=$?
    tail -1 "$OUT/pmc_packetize_$C.log"; stop_if_fatal $rc "pmc packetize $C"
  done
  python3 scripts/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"; cat "$OUT/pmc_traffic_c1.json" "$OUT/pmc_traffic_c2.json"
fi
if [ "${REQ:-1}" = 1 ]; then
  # the packetizer against the copy shapes: requests from the CUs to L2 and from L2 to memory
  CTR="TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  echo "== pmc requests: packetizer"
  timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/pmc_req_packetize" -o pmc --output-format csv -- \
    python3 scripts/run_workload.py packetize 3 > "$OUT/pmc_req_packetize.log" 2>&1; rc=$?
  tail -1 "$OUT/pmc_req_packetize.log"; stop_if_fatal $rc "pmc req packetize"
  echo "== pmc requests: copy shapes"
  COPY_SHIFT=1 timeout -s KILL 120 rocprofv3 --pmc $CTR -d "$OUT/pmc_req_copy" -o pmc --output-format csv -- \
    ./scripts/_build/copybench > "$OUT/pmc_req_copy.log" 2>&1; rc=$?
  tail -1 "$OUT/pmc_req_copy.log"; stop_if_fatal $rc "pmc req copy"
fi
echo "== done"
