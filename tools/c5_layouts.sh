set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYTEST_FILES=tests/test_gpu.py PYTEST_K="fd or skip" bash tools/gpu.sh tests || exit 1
for i in 1 2; do
  timeout -k 10 120 python bench.py --config 5 > gpurun_out/c5_l2_$i.json 2>/dev/null || exit 1
  MJHIP_FD_NOACCSKIP=1 timeout -k 10 120 python bench.py --config 5 > gpurun_out/c5_l1_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/c5_l*.json; do echo $f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'])"); done
bash tools/gpu.sh c5trace
