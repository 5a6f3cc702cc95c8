#!/bin/bash
# advection parity tests + the two solver timings + a kernel-trace profile
# usage (through gpurun): bash tools/gpu_adv.sh <tag>
set -o pipefail
tag=${1:?tag}
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_advection.py tests/test_gpu_ref_advection.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -n 40 $out/tests.log; exit 1; }
tail -n 2 $out/tests.log
timeout -k 10 120 python -u tools/adv_loop.py > $out/adv_loop.log 2>&1 && cat $out/adv_loop.log
timeout -k 10 120 python -u tools/run_adv_large.py > $out/adv_large.log 2>&1 && grep -E "us_per_step|frac" $out/adv_large.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/adv_loop.py > $out/prof.log 2>&1
python3 - $out <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True):
    for x in list(csv.DictReader(open(f)))[:3]:
        print(x["Name"][:50], x["Calls"], x["AverageNs"])
PY
