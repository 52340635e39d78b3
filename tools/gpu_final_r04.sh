set -o pipefail
bash tools/gpu_r04.sh tests && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && bash tools/gpu_r04.sh bench c4 c5
