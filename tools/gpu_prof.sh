# rocprofv3 profile of the bench (kernel trace + stats), then HBM counters in
# separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
set -u
TAG=${1:-r1}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -k line_kat -q -p no:cacheprovider > gpurun_out/linekat.log 2>&1
echo "linekat rc=$?" >> gpurun_out/linekat.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG/fetch -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG/write -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.write.log 2>&1
echo "prof rc=$?"
