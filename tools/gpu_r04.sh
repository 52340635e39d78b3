#!/bin/bash
# Round-4 GPU steps, chosen by name: tests (a pytest -k filter in PYTEST_K), bench, c4, c5
# (config 5 under a rocprofv3 kernel trace), prof (rocprof stats of the bench + PMC passes),
# variants (tools/exp_variants.py run).
#   bash tools/gpu_r04.sh tests bench c5
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      # test failures (pytest status 1) do not stop the measurement steps; anything else
      # (a timeout, an abort, a crash) ends the call
      timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests \
        -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?
      grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1 ;;
    bench)
      timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
      cat gpurun_out/bench.json ;;
    c4)
      timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json 2>&1 || exit 1
      tail -1 gpurun_out/c4.json ;;
    c5)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 \
        --output-format csv -- python bench.py --config 5 --steps 20 --warmup 3 \
        > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
      tail -1 gpurun_out/c5.json
      find gpurun_out/prof_c5 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    c5plain)
      timeout -k 10 120 python bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/c5plain.json 2>&1 || exit 1
      tail -1 gpurun_out/c5plain.json ;;
    prof)
      bash tools/gpu_profile.sh || exit 1 ;;
    sc)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sc -o sc \
        --output-format csv -- python tools/bench_model.py slider_crank 65536 20 \
        > gpurun_out/sc.log 2>&1 || { tail -20 gpurun_out/sc.log; exit 1; }
      grep -v "^W\|^\[" gpurun_out/sc.log | tail -3
      find gpurun_out/prof_sc -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    store)
      timeout -k 10 120 tools/exp_lib/exp_store > gpurun_out/store.log 2>&1 || { cat gpurun_out/store.log; exit 1; }
      cat gpurun_out/store.log ;;
    lanes)
      timeout -k 10 600 python tools/exp_lanes.py run > gpurun_out/lanes.log 2>&1 || { tail -30 gpurun_out/lanes.log; exit 1; }
      cat gpurun_out/lanes.log ;;
    variants)
      timeout -k 10 300 python tools/exp_variants.py run > gpurun_out/variants.log 2>&1 || { tail -20 gpurun_out/variants.log; exit 1; }
      cat gpurun_out/variants.log ;;
    h100)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h100 -o h100 \
        --output-format csv -- python tools/bench_model.py humanoid100 ${H100_B:-4096} 10 \
        > gpurun_out/h100.log 2>&1 || { tail -20 gpurun_out/h100.log; exit 1; }
      grep -v "^W\|^\[" gpurun_out/h100.log | tail -3
      find gpurun_out/prof_h100 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    c4t)
      timeout -k 10 120 python tools/bench_model.py humanoid_contacts 4096 20 > gpurun_out/c4t.log 2>&1 || { tail -20 gpurun_out/c4t.log; exit 1; }
      grep -v "^W\|^\[" gpurun_out/c4t.log | tail -3 ;;
    ccdblocks)
      for w in 1 2; do for nb in 512 1024 2048 4096; do
        MJHIP_CCD_WPE=$w MJHIP_CCD_BLOCKS=$nb timeout -k 10 120 python tools/bench_model.py slider_crank 65536 20 > gpurun_out/ccdb_${w}_${nb}.log 2>&1 || { tail -20 gpurun_out/ccdb_${w}_${nb}.log; exit 1; }
        echo "wpe $w blocks $nb: $(grep 'ms per call' gpurun_out/ccdb_${w}_${nb}.log)"
      done; done ;;
    step)
      timeout -k 10 180 python tools/exp_step.py > gpurun_out/step.log 2>&1 || { tail -20 gpurun_out/step.log; exit 1; }
      cat gpurun_out/step.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
