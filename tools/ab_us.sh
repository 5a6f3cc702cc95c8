#!/bin/bash
# A/B of builds of the example user-stencil library on one box:
#   bash tools/ab_us.sh TAG LIB [LIB ...]   (SKIPTEST=1: no test run first)
# runs tests/test_gpu_user_stencil.py with the in-tree build, then the user
# stencil bench line (tools/user_stencil_bench.py) once per library, three
# rounds (the first round on a fresh box reads slow: compare rounds 1 and 2)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
if [ -z "$SKIPTEST" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_user_stencil.py > gpurun_out/$tag/tests.log 2>&1 || { tail -30 gpurun_out/$tag/tests.log; exit 1; }
  tail -1 gpurun_out/$tag/tests.log
fi
for r in 0 1 2; do
  for lib in "$@"; do
    log=gpurun_out/$tag/us_${r}_$(basename $lib .so).log
    US_LIB=$lib timeout -k 10 200 python -u tools/user_stencil_bench.py > $log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('equals_library_step'))" $log $lib
  done
done
