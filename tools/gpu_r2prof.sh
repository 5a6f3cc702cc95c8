# round-2 rocprofv3 evidence for the bench: kernel trace + stats of the full
# bench command (every kernel incl. the secondary configs), then HBM counters
# of the headline kernel in separate passes (FETCH_SIZE, WRITE_SIZE), then the
# default bench line.  $1 = tag
set -u
TAG=${1:-r2}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG/fetch -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/prof_$TAG.fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG/write -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/prof_$TAG.write.log 2>&1 || exit $?
bash tools/gpu_bench.sh $TAG
