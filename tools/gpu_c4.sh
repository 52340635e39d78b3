# config-4 iteration on the GPU box: GPU parity suite, bench per lane count, phases, rocprof
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t_gpu.log 2>&1 || exit $?
for L in 16 32; do MJHIP_COOP_LANES=$L timeout -k 10 120 python bench.py --config 4 --steps 20 --warmup 3 > gpurun_out/c4_L$L.json 2>&1 || exit $?; done
MJHIP_COOP_LANES=16 timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k_L16.json 2>&1 || exit $?
timeout -k 10 120 python tools/exp_phases.py run 4096 > gpurun_out/phase16.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o prof --output-format csv -- python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/prof_c4.log 2>&1
