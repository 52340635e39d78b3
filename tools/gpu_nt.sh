#!/bin/bash
# A/B of the headline kernel with and without streaming stores, then the parity suite and the
# config-4 line of the product build
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in nt nont; do
  lib=""
  [ $v = nont ] && lib=tools/exp_lib/libmjhip_nont.so
  MJHIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o ab \
    --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "== $v: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log | head -1)"
  python - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ab_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
  if "k_all" in r["Name"]:
    print("  ", r["Name"][:20], r["Calls"], "avg", r["AverageNs"], "min", r["MinNs"], "max", r["MaxNs"])
PY
done
echo "== pytest"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
echo "== config4"
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/c4.json
