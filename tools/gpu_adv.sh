set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_advection.py -q -p no:cacheprovider > gpurun_out/adv_tests.log 2>&1
echo "adv rc=$?" >> gpurun_out/adv_tests.log
exit 0
