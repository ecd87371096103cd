#!/bin/bash
# scripts/gpu_dist_rehearsal.sh — on a one-GPU box: the bench's RCCL path (init_process_group
# "nccl", barriers, all_reduce MAX / SUM, all_gather) at world size 1, started directly and through
# torch.distributed.run exactly as the driver starts N > 1; then --gpus 2 must refuse (exit 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --dist-rehearsal --steps 10 --warmup 2 --no-cpu > $OUT/dist_direct.json 2> $OUT/dist_direct.err; rc=$?
cat $OUT/dist_direct.json; tail -3 $OUT/dist_direct.err; [ $rc -eq 0 ] || { echo "direct rc=$rc"; exit $rc; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu --dist-rehearsal --scaling strong \
  > $OUT/dist_torchrun.json 2> $OUT/dist_torchrun.err; rc=$?
cat $OUT/dist_torchrun.json; tail -3 $OUT/dist_torchrun.err; [ $rc -eq 0 ] || { echo "torchrun rc=$rc"; exit $rc; }
timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/dist_gpus2.json 2> $OUT/dist_gpus2.err; rc=$?
cat $OUT/dist_gpus2.json; tail -2 $OUT/dist_gpus2.err; echo "--gpus 2 on this box: rc=$rc (expected 2)"
[ $rc -eq 2 ] || exit 1
echo "== rehearsal done"
