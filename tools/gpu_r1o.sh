set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_amr.py tests/test_gpu_advection.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r1o_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r1o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --n 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1o_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r1o_bench.log
