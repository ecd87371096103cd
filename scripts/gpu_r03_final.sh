set -u
TESTS=0 PMC=1 bash scripts/gpu_check.sh || exit $?
rm -rf gpurun_out/prof_rx
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rx -o run --output-format csv -- python3 scripts/probe_rx.py 20 > gpurun_out/probe_rx.jsonl 2> gpurun_out/probe_rx.err; rc=$?
cat gpurun_out/probe_rx.jsonl; case $rc in 0) ;; *) echo "probe_rx rc=$rc"; tail -3 gpurun_out/probe_rx.err; exit $rc;; esac
find gpurun_out/prof_rx -name "*kernel_stats.csv" -exec cut -c1-200 {} \;
