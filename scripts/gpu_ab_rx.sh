set -u
mkdir -p gpurun_out; : > gpurun_out/rx_ab.jsonl
for i in 1 2; do
  for b in base wl cnd; do
    ICRC_AMD_LIB=$PWD/open-rdma-driver_amd/_build_ab/libicrc_amd_$b.so timeout -k 10 200 python scripts/probe_rx.py 20 > gpurun_out/rx_one.jsonl 2>gpurun_out/rx_one.err || { tail -3 gpurun_out/rx_one.err; exit 1; }
    sed "s/^{/{\"build\": \"$b\", /" gpurun_out/rx_one.jsonl >> gpurun_out/rx_ab.jsonl
  done
done
cat gpurun_out/rx_ab.jsonl
