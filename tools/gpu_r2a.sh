# round-2 start: full GPU suite, then the default bench line
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r2a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r2a_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r2a_bench.log
