#!/bin/bash
# Adaptive-loop diagnostics (configs[2]): plain timing, library phase timers,
# bench's own secondary_host_heavy, then a rocprofv3 kernel + HIP-runtime
# trace of the loop.  usage (through gpurun): bash tools/gpu_adapt_prof.sh <tag> [pytest args...]
set -o pipefail
tag=${1:?tag}
shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $out/tests.log 2>&1 \
    || { tail -n 40 $out/tests.log; exit 1; }
  tail -n 2 $out/tests.log
fi
timeout -k 10 120 python -u tools/adapt_loop.py > $out/adapt_plain.log 2>&1 || { tail -n 20 $out/adapt_plain.log; exit 1; }
tail -n 1 $out/adapt_plain.log
ADAPT_NO_TORCH=1 timeout -k 10 120 python -u tools/adapt_loop.py > $out/adapt_notorch.log 2>&1 || { tail -n 20 $out/adapt_notorch.log; exit 1; }
tail -n 1 $out/adapt_notorch.log
DCCRGX_TIMING=1 timeout -k 10 120 python -u tools/adapt_loop.py > $out/adapt_phases.log 2>&1 || { tail -n 20 $out/adapt_phases.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 tools/adapt_loop.py > $out/prof.log 2>&1 || { tail -n 20 $out/prof.log; exit 1; }
tail -n 1 $out/prof.log
ADAPT_NO_TORCH=1 timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $out/prof_nt -o run -- \
  python3 tools/adapt_loop.py > $out/prof_nt.log 2>&1 || { tail -n 20 $out/prof_nt.log; exit 1; }
tail -n 1 $out/prof_nt.log
echo done
