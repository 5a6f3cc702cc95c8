set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_amr.py tests/test_gpu_advection.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2h_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2h_tests.log; [ $rc -eq 0 ] || exit $rc
DCCRGX_TIMING=1 timeout -k 10 300 python -u tools/prof_adapt.py 5 > gpurun_out/prof_adapt2.log 2>&1
echo "rc=$?" >> gpurun_out/prof_adapt2.log
