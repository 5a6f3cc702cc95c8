#!/bin/bash
# Kernel trace, then FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes,
# of one program (default: bench.py's neighbor_lists line); summarise with
# tools/kernel_pmc_summary.py gpurun_out/<tag> <out.json> [kernel substrings].
# usage (through gpurun): bash tools/gpu_nbr_pmc.sh <tag> [tools/<program>.py]
set -o pipefail
tag=${1:?tag}
prog=${2:-tools/run_nbr_bench.py}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 $prog > $out/trace.log 2>&1 || { tail -n 20 $out/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- \
  python3 $prog > $out/fetch.log 2>&1 || { tail -n 20 $out/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- \
  python3 $prog > $out/write.log 2>&1 || { tail -n 20 $out/write.log; exit 1; }
echo done
