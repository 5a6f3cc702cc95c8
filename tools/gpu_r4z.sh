#!/bin/bash
# round-4 closing pass: full suite + smoke + bench + profiles (gpu_full.sh), the 3.5 M-leaf adaptive loop
set -o pipefail
tag=${1:-r4z}
bash tools/gpu_full.sh $tag || exit 1
out=gpurun_out/$tag
ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_3p5M.log 2>&1 || { tail -n 20 $out/adapt_3p5M.log; exit 1; }
tail -n 2 $out/adapt_3p5M.log
