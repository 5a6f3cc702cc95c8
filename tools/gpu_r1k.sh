# Round-1 re-entry check: full GPU parity suite, smoke, default bench.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r1k_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1k_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1k_smoke.log 2>&1 && \
timeout -k 10 500 python bench.py > gpurun_out/r1k_bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/r1k_bench.log
