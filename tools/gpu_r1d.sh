set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
