#!/bin/bash
# One gpurun session: each GPU step under its own time limit; stop on any fault/abort/timeout
# (exit codes other than 0 = ok and 1 = test failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-smoke pytest bench prof}"
run() {
  local name=$1 to=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 8 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}
for s in $STEPS; do
  case $s in
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 500 python -m pytest tests -m gpu -x -q ;;
    bench)  run bench 240 python bench.py --steps 20 --warmup 5 ;;
    prof)   run prof 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o prof \
              --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu ;;
  esac
done
echo "== done"
