set -u
mkdir -p gpurun_out
for t in 1 4 8 16; do
  DCCRGX_HOST_THREADS=$t DCCRGX_TIMING=1 timeout -k 10 300 python -u tools/prof_adapt.py 8 > gpurun_out/prof_threads_$t.log 2>&1 || exit 1
done
echo done
