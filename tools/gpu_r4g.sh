#!/bin/bash
# hipMalloc-backed cache: the whole GPU suite, the runtime checks that failed
# before (system runtime without torch, torch first, rt_bisect), the
# adaptive-loop timings
set -o pipefail
out=gpurun_out/r4g; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_tests.sh r4g || exit 1
for m in init adapt keep; do
  timeout -k 10 200 python -u tools/rt_bisect.py $m > $out/rt_$m.log 2>&1 || { tail -n 20 $out/rt_$m.log; exit 1; }
  grep -c FAILED $out/rt_$m.log || true
done
timeout -k 10 300 python -u tools/host_heavy_check.py > $out/hh_none.log 2>&1 || { tail -n 20 $out/hh_none.log; exit 1; }
timeout -k 10 300 python -u tools/host_heavy_check.py torch-first > $out/hh_torch.log 2>&1 || { tail -n 20 $out/hh_torch.log; exit 1; }
tail -n 1 $out/hh_none.log | head -c 600; echo
timeout -k 10 200 python -u tools/adapt_loop.py > $out/adapt_loop.log 2>&1 || { tail -n 20 $out/adapt_loop.log; exit 1; }
tail -n 3 $out/adapt_loop.log
ADAPT_NO_TORCH=1 timeout -k 10 200 python -u tools/adapt_loop.py > $out/adapt_loop_sys.log 2>&1 || { tail -n 20 $out/adapt_loop_sys.log; exit 1; }
tail -n 3 $out/adapt_loop_sys.log
