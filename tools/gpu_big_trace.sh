#!/bin/bash
# kernel + HIP-runtime trace of the 3.5 M-leaf adaptive loop (idle-gap analysis)
set -o pipefail
out=gpurun_out/bigtr; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/adapt_loop.py > $out/log 2>&1 || { tail -n 20 $out/log; exit 1; }
tail -n 1 $out/log
