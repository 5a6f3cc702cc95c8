set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gol2d" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r1m_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1m_tests.log
[ $rc -eq 0 ] || exit $rc
SWEEP_VARIANTS=0,1,16 SWEEP_WGS=8192,16384 timeout -k 10 300 python -u tools/gol2d_sweep.py > gpurun_out/r1m_sweep.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1m_prof -o run -- \
  python3 bench.py --n 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r1m_bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/r1m_bench.log
