#!/bin/bash
# GPU-box steps, run by name in order (one gpurun call, the tree already built here):
#   bash tools/gpu.sh tests smoke bench c4 c5
# Steps
#   tests     pytest -m gpu (PYTEST_K: a -k filter; PYTEST_FILES: files instead of tests/)
#   smoke     __graft_entry__.smoke()
#   bench     the default bench line                         -> gpurun_out/bench.json
#   c4 / c5   config 4 / config 5 bench lines                 -> gpurun_out/c4.json, c5.json
#   c4trace / c5trace   config 4 / 5 under a rocprofv3 kernel trace + stats
#             -> gpurun_out/prof_c4/, prof_c5/
#   prof      rocprofv3 stats of the bench line, then the PMC passes (tools/pmc.sh)
#   pmc       the PMC passes alone (PMC_ARGS: bench arguments, default the headline)
#   pmc4      config 4's PMC passes (-> gpurun_out/pmc_traffic_c4.json)
#   model     tools/bench_model.py $MODEL $B (default humanoid100 4096) under a kernel trace
#             (SKIP=1|2: mj_inverseSkip(POS|VEL) calls)
#   store     the store-layout microbenchmark, built from tools/exp_store.hip
#   lanes / variants / step   tools/exp_lanes.py, exp_variants.py, exp_step.py
# A failing pytest (status 1) does not stop the later steps; any other failure (a timeout,
# an abort, a crash) ends the call there.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
        ${PYTEST_FILES:-tests} -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?
      grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -20
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
        > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
      cat gpurun_out/bench.json ;;
    c4)
      timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4.json \
        2> gpurun_out/c4.err || exit 1
      tail -1 gpurun_out/c4.json ;;
    c4split)                                # config 4 with the split launch on (A/B)
      MJHIP_SPLIT=1 timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 \
        > gpurun_out/c4split.json 2> gpurun_out/c4split.err || exit 1
      tail -1 gpurun_out/c4split.json ;;
    c4splittrace)
      MJHIP_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4s \
        -o c4s --output-format csv -- python bench.py --config 4 --steps 20 --warmup 3 \
        > gpurun_out/c4splittrace.json 2> gpurun_out/c4splittrace.err || exit 1
      find gpurun_out/prof_c4s -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    c5)
      timeout -k 10 180 python bench.py --config 5 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
      tail -1 gpurun_out/c5.json ;;
    c5fused)                                # layout 1 in one launch, k_fdall (A/B)
      MJHIP_FD_FUSED=1 timeout -k 10 180 python bench.py --config 5 > gpurun_out/c5fused.json \
        2> gpurun_out/c5fused.err || exit 1
      tail -1 gpurun_out/c5fused.json ;;
    c5own)
      timeout -k 10 180 python bench.py --config 5 --own-stream > gpurun_out/c5own.json \
        2> gpurun_out/c5own.err || exit 1
      tail -1 gpurun_out/c5own.json ;;
    c4trace)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 \
        --output-format csv -- python bench.py --config 4 --steps 20 --warmup 3 \
        > gpurun_out/c4trace.json 2> gpurun_out/c4trace.err || exit 1
      tail -1 gpurun_out/c4trace.json
      find gpurun_out/prof_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    c5trace)
      timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 \
        --output-format csv -- python bench.py --config 5 --steps 20 --warmup 3 \
        > gpurun_out/c5trace.json 2> gpurun_out/c5trace.err || exit 1
      tail -1 gpurun_out/c5trace.json
      find gpurun_out/prof_c5 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o prof \
        --output-format csv -- python bench.py --steps 20 --warmup 5 \
        > gpurun_out/prof_bench.log 2>&1 || exit 1
      tail -1 gpurun_out/prof_bench.log
      find gpurun_out/prof_bench -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160
      python tools/rocprof_summary.py gpurun_out/prof_bench gpurun_out/rocprof_bench.json \
        > gpurun_out/rocprof_summary.log 2>&1 || exit 1
      bash tools/pmc.sh || exit 1
      cat gpurun_out/pmc_summary.log ;;
    pmc)
      bash tools/pmc.sh || exit 1
      cat gpurun_out/pmc_summary.log ;;
    pmc4)                                   # config 4's PMC passes -> pmc_traffic_c4.json
      PMC_ARGS="--config 4 --steps 3 --warmup 1" PMC_CONFIG="4 4096" bash tools/pmc.sh || exit 1
      cat gpurun_out/pmc_summary.log ;;
    model)
      m=${MODEL:-humanoid100}
      t=$m${SKIP:+_skip$SKIP}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$t -o $t \
        --output-format csv -- python tools/bench_model.py $m ${B:-4096} ${REPS:-10} \
        > gpurun_out/model_$t.log 2>&1 || { tail -20 gpurun_out/model_$t.log; exit 1; }
      grep -v "^W\|^\[" gpurun_out/model_$t.log | tail -3
      find gpurun_out/prof_$t -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 ;;
    store)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/exp_store tools/exp_store.hip || exit 1
      timeout -k 10 120 /tmp/exp_store > gpurun_out/store.log 2>&1 || { cat gpurun_out/store.log; exit 1; }
      cat gpurun_out/store.log ;;
    lanes|variants|step)
      timeout -k 10 600 python tools/exp_$step.py run > gpurun_out/$step.log 2>&1 \
        || { tail -30 gpurun_out/$step.log; exit 1; }
      cat gpurun_out/$step.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
