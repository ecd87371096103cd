#!/bin/bash
# GPU tests, then bench.py --extra alternately with this build and a B build (B_LIB), REPS times:
# gpurun_out/extra_{new,old}_<i>.json.  Every step has its own time limit; a failure stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
B=${B_LIB:-open-rdma-driver_amd/_build_ab/libicrc_amd_old.so}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/gpu_tests_ab.log 2>&1; rc=$?
  tail -3 $OUT/gpu_tests_ab.log; [ $rc = 0 ] || exit $rc
fi
for i in $(seq ${REPS:-2}); do
  timeout -k 10 300 python bench.py --extra --no-cpu --steps 20 --warmup 3 > $OUT/extra_new_$i.json 2>$OUT/extra_new_$i.err || exit 1
  ICRC_AMD_LIB=$PWD/$B timeout -k 10 300 python bench.py --extra --no-cpu --steps 20 --warmup 3 > $OUT/extra_old_$i.json 2>$OUT/extra_old_$i.err || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/extra_*_*.json")):
    d = json.load(open(f)); ex = d["extra"]
    row = {"c1": d["roofline"]["kernel_ms"]}
    for k, v in ex.items():
        if isinstance(v, dict) and ("kernel_ms" in v or "ms" in v):
            row[k] = v.get("kernel_ms", v.get("ms"))
    print(f.split("/")[-1], json.dumps(row))
PY
