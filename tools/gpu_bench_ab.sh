set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/ab_tool.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_bench_full.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-halo-payload > gpurun_out/ab_bench_nohalo.log 2>&1 || exit 1
