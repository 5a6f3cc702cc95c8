#!/bin/bash
# pool_trim_copy variants (tools/micro/pool_trim_copy.hip): which allocations
# and which copy engine lose data
set -o pipefail
out=gpurun_out/trim; mkdir -p $out; rm -f $out/all.log
run() {
  timeout -k 10 120 "$@" > $out/one.log 2>&1 || { cat $out/one.log; exit 1; }
  cat $out/one.log >> $out/all.log
  echo "$(env | grep -E '^HSA_ENABLE_SDMA' || true) $(tail -n 1 $out/one.log)"
}
run tools/micro/pool_trim_copy 40 0 1 1 1 0
run tools/micro/pool_trim_copy 40 0 1 1 0 1
run tools/micro/pool_trim_copy 40 0 1 2 1 2
run tools/micro/pool_trim_copy 40 0 1 2 0 2
run tools/micro/pool_trim_copy 40 1 1 2 0 1
export HSA_ENABLE_SDMA=0
run tools/micro/pool_trim_copy 40 0 1 1 1 0
run tools/micro/pool_trim_copy 40 0 1 1 0 1
run tools/micro/pool_trim_copy 40 1 1 0 0 1
