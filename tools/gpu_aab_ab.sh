set -u
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/aab_pinned_$r.log 2>&1 || exit 1
  DCCRGX_PAGEABLE=1 timeout -k 10 200 python -u tools/adapt_after_big.py > gpurun_out/aab_pageable_$r.log 2>&1 || exit 1
done
