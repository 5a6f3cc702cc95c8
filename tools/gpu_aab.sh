set -u
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/aab_$r.log 2>&1 || exit 1
done
DCCRGX_TIMING=1 timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/aab_t.log 2>&1
