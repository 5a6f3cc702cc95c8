set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_poisson.py tests/test_gpu_face.py -q -p no:cacheprovider > gpurun_out/poisson_tests.log 2>&1
echo "rc=$?" >> gpurun_out/poisson_tests.log
exit 0
