set -o pipefail
out=gpurun_out/r4b; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_ref_advection.py tests/test_gpu_rccl.py tests/test_gpu_multiprocess.py tests/test_gpu_amr.py tests/test_gpu_streams.py tests/test_facade.py tests/test_gpu_ref_gol.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -n 40 $out/tests.log; exit 1; }
tail -n 2 $out/tests.log
timeout -k 10 120 python -u tools/adv_loop.py > $out/adv_loop.log 2>&1 && cat $out/adv_loop.log
timeout -k 10 120 python -u tools/run_adv_large.py > $out/adv_large.log 2>&1 && cat $out/adv_large.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/adv_loop.py > $out/prof.log 2>&1
find $out/prof -name '*kernel_stats.csv' | head -n 3
