#!/bin/bash
# advection kernel occupancy sweep (DCCRGX_ADV_WPE) on both solver timings
set -o pipefail
out=gpurun_out/${1:?tag}; mkdir -p $out
for w in 1 5 6 8; do
  echo "WPE=$w"
  DCCRGX_ADV_WPE=$w timeout -k 10 120 python -u tools/adv_loop.py 2>&1 | grep cells
  DCCRGX_ADV_WPE=$w timeout -k 10 120 python -u tools/run_adv_large.py 2>&1 | grep -E "us_per_step"
done > $out/sweep.log
cat $out/sweep.log
