#!/bin/bash
# the whole -m gpu suite (optionally a subset: pytest args), then optional extra script
# usage (through gpurun): bash tools/gpu_tests.sh <tag> [pytest targets...]
set -o pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
targets=${@:-tests}
timeout -k 10 900 python -u -m pytest $targets -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -n 60 $out/gpu_tests.log; exit 1; }
tail -n 2 $out/gpu_tests.log
