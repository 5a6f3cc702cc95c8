set -u
mkdir -p gpurun_out
DCCRGX_TIMING=1 timeout -k 10 300 python -u tools/prof_adapt.py 20 > gpurun_out/prof_adapt.log 2>&1
echo "rc=$?" >> gpurun_out/prof_adapt.log
