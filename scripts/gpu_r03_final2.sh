#!/bin/bash
# Round-3 final measurement pass: every GPU test, smoke, bench (plain and under torchrun as one
# rank), rocprofv3 stats of plain bench, FETCH_SIZE / WRITE_SIZE for roofline.traffic, bench --extra,
# C2 HBM traffic on the default hybrid launch.  Every GPU step under its own time limit; a fatal
# exit (124/134/137/139) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "FATAL: $2 exited $1"; exit "$1";; esac; }
STEPS=tests,smoke bash scripts/gpu_session.sh || exit $?
TESTS=0 PMC=1 bash scripts/gpu_check.sh || exit $?
echo "== torchrun, one rank"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu > $OUT/bench_trun.json 2> $OUT/bench_trun.err; rc=$?
tail -c 600 $OUT/bench_trun.json; echo; fatal $rc torchrun
echo "== extra"
STEPS=extra bash scripts/gpu_session.sh || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmcc2f_$C
  timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmcc2f_$C -o pmc --output-format csv -- python3 scripts/run_workload.py c2 3 \
    > $OUT/pmcc2f_$C.log 2>&1; rc=$?; tail -1 $OUT/pmcc2f_$C.log; fatal $rc "pmc c2 $C"
done
python3 - <<'PY' | tee $OUT/pmc_c2_final.txt
import csv, glob, collections
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(float); disp = collections.defaultdict(set)
    for path in glob.glob(f"gpurun_out/pmcc2f_{C}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            if "icrc" not in k or "synth" in k:
                continue
            acc[k] += float(r["Counter_Value"]); disp[k].add(r.get("Dispatch_Id"))
    for k, v in acc.items():
        print(C, k, "dispatches", len(disp[k]), "KB per dispatch", round(v / max(1, len(disp[k])), 1))
PY
echo "== done"
