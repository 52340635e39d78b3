#!/bin/bash
# config-4 iteration on the GPU box: GPU parity suite, bench lines, phases, rocprof of config 4
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
timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k.json 2>&1 || exit 1
tail -1 gpurun_out/c4_64k.json
echo "== phases (tools/exp_lib build must match the tree)"
timeout -k 10 120 python tools/exp_phases.py run 4096 > gpurun_out/phase16.log 2>&1 || exit 1
cat gpurun_out/phase16.log
for cq in 1 2; do
  if [ -f tools/exp_lib/libmjhip_phase_cq$cq.so ]; then
    echo "-- $cq lane(s) per contact"
    PHASE_CQ=$cq timeout -k 10 120 python tools/exp_phases.py run 4096 > gpurun_out/phase16_cq$cq.log 2>&1 || exit 1
    grep -A6 "k_constraint_coop\|per contact" gpurun_out/phase16_cq$cq.log | grep -v generic
  fi
done
echo "== rocprof config4"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o prof --output-format csv -- python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/prof_c4.log 2>&1 || exit 1
find gpurun_out/prof_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
echo "== slider_crank (config-1 model) straight-line kernel"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sc -o sc --output-format csv -- python tools/bench_model.py slider_crank 65536 20 > gpurun_out/sc.log 2>&1 || exit 1
grep "evals/s" gpurun_out/sc.log
find gpurun_out/prof_sc -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -5
