#!/bin/bash
# config 5 bench line and its rocprof summary only
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu \
  -k "fd or linear_system" > gpurun_out/pytest_fd.log 2>&1 || { tail -30 gpurun_out/pytest_fd.log; exit 1; }
tail -1 gpurun_out/pytest_fd.log
timeout -k 10 180 python bench.py --config 5 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail gpurun_out/c5.err; exit 1; }
tail -1 gpurun_out/c5.json | cut -c1-300
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/prof_c5.log 2>&1 || exit 1
find gpurun_out/prof_c5 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-120
