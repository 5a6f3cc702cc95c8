# bench with the secondary configs, then a rocprof kernel-trace of the same run
set -u
TAG=r1g
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_$TAG.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/bench_$TAG.log
exit 0
