mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/skew_tests.log 2>&1; rc=$?; tail -2 gpurun_out/skew_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
B_LIB=open-rdma-driver_amd/_build_ab/old/libicrc_amd.so VARIANTS=-1 JOBS=C1,C2,S316,C2k REPS=3 bash scripts/gpu_ab_lib.sh > gpurun_out/skew_ab_lib.log 2>&1 || { tail -5 gpurun_out/skew_ab_lib.log; exit 1; }
timeout -k 10 300 python scripts/probe_oct_balance.py > gpurun_out/oct_balance_skew.jsonl 2> gpurun_out/oct_balance_skew.err; rc=$?; cut -c1-400 gpurun_out/oct_balance_skew.jsonl; exit $rc
