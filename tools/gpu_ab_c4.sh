#!/bin/bash
# config-4 A/B of the cooperative kernel's lanes per contact (phase-timing builds: their marks
# cost the same in every variant), then the headline profile (tools/gpu_profile.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" _cq1 _cq2; do
  lib=tools/exp_lib/libmjhip_phase$v.so
  [ -f $lib ] || continue
  MJHIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab$v -o ab \
    --output-format csv -- python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/ab$v.log 2>&1 || exit 1
  echo "== variant ${v:-_cq4}: $(grep -o '"value": [0-9.]*' gpurun_out/ab$v.log)"
  python - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/ab{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
  if "coop" in r["Name"] or "k_all" in r["Name"]:
    print("  ", r["Name"][:28], r["Calls"], "avg", r["AverageNs"], "max", r["MaxNs"])
PY
done
bash tools/gpu_profile.sh
