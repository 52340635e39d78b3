#!/bin/bash
# GPU parity suite + the bench line (round 3 check). Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
grep -h "convex pairs:\|slider_crank:" gpurun_out/pytest_gpu.log || true
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
echo "== config4"
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
tail -1 gpurun_out/c4.json
