#!/bin/bash
# advection kernel variants: global vs buffer loads x waves per SIMD, both sizes, then the parity tests (default build)
set -o pipefail
out=gpurun_out/advl; mkdir -p $out; rm -f $out/sweep.log
for buf in ${ADV_BUFS:-0 1}; do for wpe in ${ADV_WPES:-4 5}; do
  echo "buf=$buf wpe=$wpe" >> $out/sweep.log
  DCCRGX_ADV_BUF=$buf DCCRGX_ADV_WPE=$wpe timeout -k 10 120 python -u tools/adv_loop.py >> $out/sweep.log 2>&1 || { tail -n 20 $out/sweep.log; exit 1; }
  DCCRGX_ADV_BUF=$buf DCCRGX_ADV_WPE=$wpe timeout -k 10 120 python -u tools/run_adv_large.py > $out/large.log 2>&1 || { tail -n 20 $out/large.log; exit 1; }
  grep -E "us_per_step|frac" $out/large.log >> $out/sweep.log
done; done
cat $out/sweep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_ref_advection.py tests/test_gpu_amr.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -n 40 $out/tests.log; exit 1; }
tail -n 2 $out/tests.log
