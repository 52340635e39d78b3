#!/bin/bash
# Round-end profile of the headline bench on the GPU box: rocprofv3 kernel stats of the
# default bench line, then the PMC traffic passes (tools/pmc.sh) and their summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== rocprof bench"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o prof \
  --output-format csv -- python bench.py --steps 20 --warmup 5 > gpurun_out/prof_bench.log 2>&1 || exit 1
tail -1 gpurun_out/prof_bench.log
find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
python tools/rocprof_summary.py gpurun_out/prof_bench gpurun_out/rocprof_bench.json > gpurun_out/rocprof_summary.log 2>&1 || exit 1
echo "== pmc"
bash tools/pmc.sh || exit 1
cat gpurun_out/pmc_summary.log
