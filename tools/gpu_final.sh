#!/bin/bash
# end-of-round evidence on the GPU box: the whole GPU suite, the bench lines of configs 1, 4
# (4,096 and 65,536) and 5, the rocprof summary of the default bench, and the straight-line
# kernel of a model that runs through the tendon and discrete passes
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
echo "== config 4 / 5"
timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
tail -1 gpurun_out/c4.json
timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k.json 2>&1 || exit 1
tail -1 gpurun_out/c4_64k.json
timeout -k 10 180 python bench.py --config 5 > gpurun_out/c5.json 2>&1 || exit 1
tail -1 gpurun_out/c5.json
echo "== rocprof bench"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench.log 2>&1 || exit 1
find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
echo "== passes: spatial tendon + INVDISCRETE model"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_passes -o passes --output-format csv -- python tools/bench_model.py tools/passes_model.xml 65536 20 > gpurun_out/passes.log 2>&1 || exit 1
grep "evals/s" gpurun_out/passes.log
find gpurun_out/prof_passes -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
