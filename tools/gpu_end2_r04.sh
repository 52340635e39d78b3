#!/bin/bash
# after the exact-unit split: the full GPU suite, smoke, bench, slider_crank parity prints
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_final_r04.sh || exit 1
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
  tests/test_convex_gpu.py tests/test_gpu.py -k "slider or convex" > gpurun_out/sc_prints.log 2>&1 || exit 1
grep -E "slider|convex pairs|passed|failed" gpurun_out/sc_prints.log | cut -c1-300
timeout -k 10 120 python tools/bench_model.py slider_crank 65536 20 > gpurun_out/sc_end.log 2>&1 || exit 1
grep "ms per call" gpurun_out/sc_end.log
