#!/bin/bash
# Round measurement on the GPU box: GPU parity suite, the bench line, its rocprofv3 kernel
# stats, PMC traffic passes, configs 4 and 5. Outputs under gpurun_out/ (copied to
# profiles/<round>/ afterwards). Every GPU step has its own time limit; the first failure ends.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || exit $?
step bench
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o prof \
  --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu \
  > gpurun_out/prof_bench.log 2>&1 || exit $?
step pmc
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
step config4
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit $?
step config5
timeout -k 10 180 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/c5.json 2>&1 || exit $?
echo done
