# full GPU suite (log under gpurun_out/$1_tests.log); stops at the first failure
set -u
TAG=${1:-t}
shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_tests.log; exit $rc
