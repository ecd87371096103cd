set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests3.log; [ $rc = 0 ] || exit $rc
ROUNDS=5 timeout -k 10 300 python scripts/ab_variants.py -1,17,19 > gpurun_out/ab_prio.jsonl 2>gpurun_out/ab_prio.err || exit 1
cat gpurun_out/ab_prio.jsonl
for i in 1 2; do
  timeout -k 10 300 python bench.py --extra --no-cpu --steps 20 --warmup 3 > gpurun_out/extra_new_$i.json 2>gpurun_out/extra_new_$i.err || exit 1
  ICRC_AMD_LIB=$PWD/open-rdma-driver_amd/_build_ab/libicrc_amd_old.so timeout -k 10 300 python bench.py --extra --no-cpu --steps 20 --warmup 3 > gpurun_out/extra_old_$i.json 2>gpurun_out/extra_old_$i.err || exit 1
done
echo done
