set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_amr.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/amr_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/amr_tests.log
