#!/bin/bash
# neighbor-list query kernels (bench.py's neighbor_lists line): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes.
# usage (through gpurun): bash tools/gpu_nbr_pmc.sh <tag>
set -o pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 tools/run_nbr_bench.py > $out/nbr_trace.log 2>&1 || { tail -n 20 $out/nbr_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
  python3 tools/run_nbr_bench.py > $out/nbr_fetch.log 2>&1 || { tail -n 20 $out/nbr_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
  python3 tools/run_nbr_bench.py > $out/nbr_write.log 2>&1 || { tail -n 20 $out/nbr_write.log; exit 1; }
echo done
