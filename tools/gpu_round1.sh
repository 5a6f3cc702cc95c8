set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/bench.log
fi
exit 0
