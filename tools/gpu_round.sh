#!/bin/bash
# Round-end GPU evidence: parity suite, bench lines (headline, config 4 at 4,096 and 65,536,
# config 5), then the headline rocprof summary and PMC traffic (tools/gpu_profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest"
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
grep -h "convex pairs:\|slider_crank:\|geom distance sensors:" gpurun_out/pytest_gpu.log || true
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bench.json | head -1
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/c4.json | head -1
timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k.json 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/c4_64k.json | head -1
timeout -k 10 200 python bench.py --config 5 > gpurun_out/c5.json 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/c5.json | head -1
bash tools/gpu_profile.sh
