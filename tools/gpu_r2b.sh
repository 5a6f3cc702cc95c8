# round 2 re-entry: full GPU suite, stencil variant sweep (incl. wave-independent k_gol26w), default bench
set -u
mkdir -p gpurun_out
bash tools/gpu_tests.sh r2b || exit $?
SWEEP_VARIANTS=841,904,906,908,912,916,8412 SWEEP_WGS=8192,32768 SWEEP_ROUNDS=3 \
  timeout -k 10 400 python -u tools/gol_sweep.py > gpurun_out/r2b_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc" >> gpurun_out/r2b_sweep.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench.sh r2b
