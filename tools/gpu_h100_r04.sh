#!/bin/bash
# humanoid100 row-span measurements: the parity tests, then bench_model at two batches
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
PYTEST_K="sparse or humanoid100 or dropin or adapter or abi or slider" bash tools/gpu_r04.sh tests || exit 1
for b in 4096 16384; do
  H100_B=$b bash tools/gpu_r04.sh h100 || exit 1
  cp gpurun_out/h100.log gpurun_out/h100_b$b.log
  cp gpurun_out/prof_h100/h100_kernel_stats.csv gpurun_out/h100_b${b}_kernel_stats.csv
done
