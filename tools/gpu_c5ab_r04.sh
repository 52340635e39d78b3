#!/bin/bash
# config 5 A/B: the FD expansion split around the position-stage kernel (default) vs one
# expansion ahead of it (MJHIP_FD_NOSPLIT=1), three runs each, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
PYTEST_K="inverse_fd" bash tools/gpu_r04.sh tests || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/c5_split_$r.json 2>&1 || exit 1
  MJHIP_FD_NOSPLIT=1 timeout -k 10 120 python bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/c5_nosplit_$r.json 2>&1 || exit 1
  echo "run $r: split $(tail -1 gpurun_out/c5_split_$r.json | cut -c1-130)"
  echo "run $r: nosplit $(tail -1 gpurun_out/c5_nosplit_$r.json | cut -c1-130)"
done
