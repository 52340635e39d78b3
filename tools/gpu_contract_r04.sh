#!/bin/bash
# A/B: the product library vs the constraint unit compiled without contraction
# (tools/exp_contract.py): convex/reference-model parity fractions, config 4, slider_crank
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in product ccoff; do
  if [ $v = ccoff ]; then export MJHIP_LIB=tools/exp_lib/libmjhip_ccoff.so; fi
  timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread \
    tests/test_convex_gpu.py tests/test_reference_model_gpu.py > gpurun_out/contract_$v.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
  grep -E "convex pairs|reference model|slider_crank|passed|failed" gpurun_out/contract_$v.log | cut -c1-330
  timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4_$v.json 2>&1 || exit 1
  echo "$v c4: $(tail -1 gpurun_out/c4_$v.json | cut -c1-110)"
  timeout -k 10 120 python tools/bench_model.py slider_crank 65536 20 > gpurun_out/sc_$v.log 2>&1 || exit 1
  echo "$v sc: $(grep 'ms per call' gpurun_out/sc_$v.log)"
done
