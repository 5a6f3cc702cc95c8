#!/bin/bash
# whole suite, then the adaptive loop at 218k and 3.5 M leaves with a kernel trace of the latter
set -o pipefail
bash tools/gpu_tests.sh r4n || exit 1
out=gpurun_out/r4n
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u tools/adapt_loop.py > $out/adapt.log 2>&1 || { tail -n 20 $out/adapt.log; exit 1; }
tail -n 1 $out/adapt.log
ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_big.log 2>&1 || { tail -n 20 $out/adapt_big.log; exit 1; }
tail -n 1 $out/adapt_big.log
ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $out/big_prof -o run -- python3 tools/adapt_loop.py > $out/big_prof.log 2>&1 || { tail -n 20 $out/big_prof.log; exit 1; }
echo done
