#!/bin/bash
# adaptive loop phases at 218k and 3.5 M leaves (synchronised per phase) and the library's phase laps
set -o pipefail
out=gpurun_out/aseg; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ADAPT_SEG=1 timeout -k 10 200 python -u tools/adapt_loop.py > $out/small.log 2>&1 || { tail -n 20 $out/small.log; exit 1; }
tail -n 2 $out/small.log
ADAPT_SEG=1 ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/big.log 2>&1 || { tail -n 20 $out/big.log; exit 1; }
tail -n 2 $out/big.log
DCCRGX_TIMING=1 ADAPT_STEPS=8 ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/big_timing.log 2>&1 || { tail -n 20 $out/big_timing.log; exit 1; }
tail -n 1 $out/big_timing.log
