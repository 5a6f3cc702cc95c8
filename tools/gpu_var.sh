set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_variable.py -q -p no:cacheprovider -x > gpurun_out/var_tests.log 2>&1
echo "var rc=$?" >> gpurun_out/var_tests.log
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
exit 0
