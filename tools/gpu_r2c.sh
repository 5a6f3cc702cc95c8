# AMR/advection/mapping parity after the override_unrefines and mapping-kernel changes,
# mapping sweep, HBM read/write-mix ceiling, adaptive phase timers
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_amr.py tests/test_gpu_advection.py tests/test_gpu_parity.py -k "amr or advect or adapt or mapping" \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/map_sweep.py > gpurun_out/r2c_map.log 2>&1 || exit $?
timeout -k 10 200 ./tools/micro/bw_mix 8 > gpurun_out/r2c_bwmix.log 2>&1 || exit $?
DCCRGX_TIMING=1 timeout -k 10 300 python -u tools/prof_adapt.py 5 > gpurun_out/r2c_adapt.log 2>&1
echo "adapt rc=$?" >> gpurun_out/r2c_adapt.log
