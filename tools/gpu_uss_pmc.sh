#!/bin/bash
# SQ / TA / TCC counters of the user-stencil game of life at 2048^3, one pass per counter group
set -o pipefail
out=gpurun_out/usspmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" \
           "TA_BUSY_avr TA_BUSY_max TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out/p$i -o run -- python3 tools/user_stencil_bench.py > $out/p$i.log 2>&1
  rc=$?
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then tail -n 20 $out/p$i.log; exit 1; fi
  [ $rc -ne 0 ] && { echo "group $i failed rc=$rc"; tail -n 3 $out/p$i.log; }
done
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
res = collections.defaultdict(list)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_user_staged" in r["Kernel_Name"]:
            res[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(res.items()):
    print(k, sum(v) / len(v))
PY
