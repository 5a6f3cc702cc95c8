set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -k "mapping" -q -p no:cacheprovider > gpurun_out/r1i_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r1i_tests.log
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r1i_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r1i_tests.log
exit 0
