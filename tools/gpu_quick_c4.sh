set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu -k "coop or contact or c4 or elliptic or touch" > gpurun_out/pytest_quick.log 2>&1 || { tail -20 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/c4.json | head -1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o prof --output-format csv -- python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/prof_c4.log 2>&1 || exit 1
python3 -c "
import csv, glob
f = glob.glob('gpurun_out/prof_c4/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
  print(r['Name'][:40], r['Calls'], r['AverageNs'], r['MaxNs'])
"
timeout -k 10 120 python tools/exp_phases.py run 4096 > gpurun_out/phase16.log 2>&1 || exit 1
grep -A6 "k_constraint_coop" gpurun_out/phase16.log
