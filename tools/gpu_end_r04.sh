#!/bin/bash
# round-end validation at HEAD: profiles of the shipped kernel (placed where bench.py finds
# them), the full GPU suite, smoke, bench, configs 4 and 5, slider_crank, parity prints
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_r04.sh prof || exit 1
cp gpurun_out/pmc_traffic.json gpurun_out/rocprof_bench.json profiles/r04/ || exit 1
bash tools/gpu_final_r04.sh || exit 1
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
  tests/test_convex_gpu.py tests/test_reference_model_gpu.py > gpurun_out/parity_prints.log 2>&1 || exit 1
grep -E "convex pairs|reference model|slider_crank|passed|failed" gpurun_out/parity_prints.log | cut -c1-330
timeout -k 10 120 python tools/bench_model.py slider_crank 65536 20 > gpurun_out/sc_end.log 2>&1 || exit 1
grep "ms per call" gpurun_out/sc_end.log
