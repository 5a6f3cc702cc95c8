#!/bin/bash
# round-4 pass: the full GPU suite + smoke + bench + profiles (gpu_full.sh),
# the advection timings (gpu_adv.sh), and the pool-trim reproducer
# usage (through gpurun): bash tools/gpu_r4.sh <tag>
set -o pipefail
tag=${1:?tag}
bash tools/gpu_full.sh $tag || exit 1
bash tools/gpu_adv.sh ${tag}_adv || exit 1
out=gpurun_out/$tag
for args in "200 1 1" "200 1 0" "200 0 1"; do
  timeout -k 10 120 tools/micro/pool_trim_copy $args >> $out/pool_trim.log 2>&1 || { tail -n 5 $out/pool_trim.log; exit 1; }
done
cat $out/pool_trim.log | tail -n 3
