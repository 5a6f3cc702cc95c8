set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  SWEEP_WGS=2048,8192,32768 timeout -k 10 600 python tools/gol_sweep.py > gpurun_out/sweep.log 2>&1
  echo "sweep rc=$?" >> gpurun_out/sweep.log
fi
exit 0
