set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gol" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r1l_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1l_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gol2d_sweep.py > gpurun_out/r1l_sweep.log 2>&1
echo "sweep rc=$?" >> gpurun_out/r1l_sweep.log
