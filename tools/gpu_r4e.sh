#!/bin/bash
# mixed-level list build parity + PMC of the neighbor benchmark + pool-trim variants
set -o pipefail
out=gpurun_out/r4e; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_explicit.py tests/test_gpu_parity.py tests/test_gpu_amr.py tests/test_gpu_face.py tests/test_gpu_gol_amr.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -n 40 $out/tests.log; exit 1; }
tail -n 2 $out/tests.log
bash tools/gpu_nbr_pmc.sh r4e_nbr || exit 1
grep -E "initialize_s|\"ms\"" gpurun_out/r4e_nbr/trace.log | head -5
for args in "100 0 1 0 0" "100 1 1 1 0" "100 1 1 0 1" "100 1 0 0 0"; do
  timeout -k 10 120 tools/micro/pool_trim_copy $args > $out/trim.tmp 2>&1 || { cat $out/trim.tmp; exit 1; }
  tail -n 1 $out/trim.tmp | tee -a $out/pool_trim.log
done
TL=$(python3 -c "import os,torch;print(os.path.dirname(torch.__file__)+'/lib')")
LD_LIBRARY_PATH=$TL timeout -k 10 120 tools/micro/pool_trim_copy 100 1 1 0 0 > $out/trim.tmp 2>&1 || { cat $out/trim.tmp; exit 1; }
echo "torch runtime ($TL):" | tee -a $out/pool_trim.log; tail -n 1 $out/trim.tmp | tee -a $out/pool_trim.log
