# default bench line -> gpurun_out/$1_bench.log
set -u
TAG=${1:-b}
shift || true
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/${TAG}_bench.log; exit $rc
