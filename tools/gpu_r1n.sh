set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_explicit.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r1n_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1n_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1n_prof -o run -- \
  python3 bench.py --n 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1n_bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/r1n_bench.log
