# stencil variant sweep (one process, interleaved) after the variant parity tests
set -u
TAG=${1:-sw}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "variants" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_VARIANTS=${SWEEP_VARIANTS:-841,8412,84111,84121,4412,44121} SWEEP_WGS=${SWEEP_WGS:-8192,16384} SWEEP_ROUNDS=3 \
  timeout -k 10 600 python -u tools/gol_sweep.py > gpurun_out/${TAG}_sweep.log 2>&1
echo "sweep rc=$?" >> gpurun_out/${TAG}_sweep.log
