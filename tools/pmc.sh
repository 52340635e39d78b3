#!/bin/bash
# PMC passes over a short bench run (GPU box). Each counter group in its own rocprofv3 run
# (kernel-trace only alongside --pmc); outputs under gpurun_out/pmc_<n>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for group in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" "FETCH_SIZE" \
             "WRITE_SIZE"; do
  n=$((n+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $group -d gpurun_out/pmc_$n -o pmc \
    --output-format csv -- python bench.py ${PMC_ARGS:---steps 3 --warmup 1 --no-cpu} \
    > gpurun_out/pmc_$n.log 2>&1
  rc=$?
  echo "pmc pass $n ($group) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
if [ -n "${PMC_CONFIG:-}" ]; then        # e.g. PMC_CONFIG="4 4096" with PMC_ARGS="--config 4 ..."
  python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic_c4.json $PMC_CONFIG \
    > gpurun_out/pmc_summary.log 2>&1
else
  python tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.log 2>&1
fi
exit $?
