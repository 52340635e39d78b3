export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu -k "coop or status_bits or config4 or config3 or config2_parity or full_size" > gpurun_out/t2.log 2>&1 || exit $?
for L in 16 8 0; do MJHIP_COOP_LANES=$L timeout -k 10 120 python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/c4_L$L.log 2>&1 || exit $?; done
MJHIP_COOP_LANES=16 timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k_L16.log 2>&1 || exit $?
MJHIP_COOP_LANES=8 timeout -k 10 120 python bench.py --config 4 --config-batch 65536 --steps 5 --warmup 2 > gpurun_out/c4_64k_L8.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4b -o prof --output-format csv -- python bench.py --config 4 --steps 10 --warmup 3 > gpurun_out/prof_c4b.log 2>&1
