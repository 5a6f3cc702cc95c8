#!/bin/bash
# the library's phase laps of the 218k-leaf adaptive loop, and the API census of the same run
set -o pipefail
out=gpurun_out/asm; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
DCCRGX_TIMING=1 ADAPT_STEPS=12 timeout -k 10 200 python -u tools/adapt_loop.py > $out/timing.log 2>&1 || { tail -n 20 $out/timing.log; exit 1; }
tail -n 1 $out/timing.log
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/adapt_loop.py > $out/prof.log 2>&1 || { tail -n 20 $out/prof.log; exit 1; }
echo done
