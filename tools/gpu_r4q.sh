#!/bin/bash
# whole suite, then the adaptive loop at 218k and 3.5 M leaves, the advection solver alone at 183k
set -o pipefail
bash tools/gpu_tests.sh r4q || exit 1
out=gpurun_out/r4q
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u tools/adapt_loop.py > $out/adapt.log 2>&1 || { tail -n 20 $out/adapt.log; exit 1; }
tail -n 1 $out/adapt.log
ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_big.log 2>&1 || { tail -n 20 $out/adapt_big.log; exit 1; }
tail -n 1 $out/adapt_big.log
timeout -k 10 200 python -u tools/adv_small.py > $out/adv_small.log 2>&1 || { tail -n 20 $out/adv_small.log; exit 1; }
tail -n 2 $out/adv_small.log
