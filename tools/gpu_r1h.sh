set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_poisson.py tests/test_gpu_advection.py -q -p no:cacheprovider > gpurun_out/r1h_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r1h_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1h/trace -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r1h.bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/r1h_tests.log
exit 0
