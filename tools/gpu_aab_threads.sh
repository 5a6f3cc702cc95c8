set -u
mkdir -p gpurun_out
for t in 1 2 4 16; do
  DCCRGX_HOST_THREADS=$t DCCRGX_TIMING=1 timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/aab_th$t.log 2>&1 || exit 1
done
