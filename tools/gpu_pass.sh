#!/bin/bash
# One GPU pass, steps chosen on the command line (each under its own time
# limit; the pass stops at the first failing step):
#   bash tools/gpu_pass.sh TAG STEP [STEP ...]
# steps:
#   tests[=PYTEST_ARGS]  pytest -m gpu (default: the whole GPU suite) -> TAG/tests.log
#   smoke                __graft_entry__.smoke()                     -> TAG/smoke.log
#   bench                bench.py --steps 20 --warmup 3               -> TAG/bench.log
#   prof                 rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the
#                        headline (summarize: python tools/summarize_prof.py TAG/prof ...)
#   us                   tools/user_stencil_bench.py (+ --stats)      -> TAG/us.log, TAG/us_prof/
#   uspmc                FETCH/WRITE + SQ passes of the user stencil  -> TAG/uspmc_*/
#   adapt / adaptbig     tools/adapt_loop.py at 218k / 3.5 M leaves   -> TAG/adapt*.log
#   advlarge             tools/run_adv_large.py                        -> TAG/adv_large.log
#   adaptsplit           adapt_grid split into its parts; sync phase timers -> TAG/adapt_*split*.log
#   adapttrace           3.5 M-leaf adaptive loop: phases, trace, idle gaps -> TAG/adapt_*
#   py=SCRIPT            python -u SCRIPT                              -> TAG/<script>.log
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
fail() { echo "step $1 failed rc=$2"; tail -n 30 "$3"; exit 1; }
for step in "$@"; do
  case $step in
    tests*)
      args=${step#tests}; args=${args#=}; [ -z "$args" ] && args="tests"
      timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $args > $out/tests.log 2>&1 || fail tests $? $out/tests.log
      tail -n 2 $out/tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1 || fail smoke $? $out/smoke.log
      tail -n 1 $out/smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > $out/bench.log 2>&1 || fail bench $? $out/bench.log
      tail -n 1 $out/bench.log | cut -c1-600 ;;
    prof)
      # kernel trace + stats, then FETCH_SIZE / WRITE_SIZE in passes of their own
      # (the layout tools/summarize_prof.py reads: prof/trace, prof/fetch, prof/write)
      q="--no-secondary --no-halo-payload --no-cpu-baseline --no-check"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 $q > $out/prof_trace.log 2>&1 || fail prof_trace $? $out/prof_trace.log
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/prof/fetch -o run -- python3 bench.py --steps 3 --warmup 1 $q > $out/prof_fetch.log 2>&1 || fail prof_fetch $? $out/prof_fetch.log
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/prof/write -o run -- python3 bench.py --steps 3 --warmup 1 $q > $out/prof_write.log 2>&1 || fail prof_write $? $out/prof_write.log ;;
    us)
      timeout -k 10 300 python -u tools/user_stencil_bench.py > $out/us.log 2>&1 || fail us $? $out/us.log
      cat $out/us.log | cut -c1-1500
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/us_prof -o run -- python3 tools/user_stencil_bench.py > $out/us_prof.log 2>&1 || fail us_prof $? $out/us_prof.log ;;
    uspmc)
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out/uspmc_$i -o run -- python3 tools/user_stencil_bench.py > $out/uspmc_$i.log 2>&1 || fail uspmc_$i $? $out/uspmc_$i.log
      done ;;
    adapt)
      timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt.log 2>&1 || fail adapt $? $out/adapt.log
      tail -n 2 $out/adapt.log ;;
    adaptbig)
      ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_3p5M.log 2>&1 || fail adaptbig $? $out/adapt_3p5M.log
      tail -n 2 $out/adapt_3p5M.log ;;
    adapttrace)
      # the 3.5 M-leaf adaptive loop: library phase timers, then a kernel +
      # HIP-runtime trace (no counters) and its device-idle report
      ADAPT_N=1600 ADAPT_REL=0.006 DCCRGX_TIMING=1 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_big_phases.log 2>&1 || fail adapt_phases $? $out/adapt_big_phases.log
      tail -n 2 $out/adapt_big_phases.log
      ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/adapt_trace -o run -- python3 tools/adapt_loop.py > $out/adapt_trace.log 2>&1 || fail adapt_trace $? $out/adapt_trace.log
      python3 tools/idle_gaps.py $out/adapt_trace > $out/adapt_gaps.txt 2>&1; tail -n 25 $out/adapt_gaps.txt ;;
    adaptsmall)
      # configs[2]'s 218k-leaf adaptive loop: split timing, phase timers that
      # wait per lap, then a kernel + HIP-runtime trace and its census
      timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_plain.log 2>&1 || fail adapt_plain $? $out/adapt_plain.log
      tail -n 1 $out/adapt_plain.log
      ADAPT_HOST_SETS=1 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_host_sets.log 2>&1 || fail adapt_host_sets $? $out/adapt_host_sets.log
      tail -n 1 $out/adapt_host_sets.log
      ADAPT_SEG=2 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_split.log 2>&1 || fail adapt_split $? $out/adapt_split.log
      tail -n 3 $out/adapt_split.log
      DCCRGX_TIMING=2 ADAPT_STEPS=8 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_sync_phases.log 2>&1 || fail adapt_sync_phases $? $out/adapt_sync_phases.log
      timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/adapt_trace -o run -- python3 tools/adapt_loop.py > $out/adapt_trace.log 2>&1 || fail adapt_trace $? $out/adapt_trace.log
      tail -n 2 $out/adapt_trace.log
      python3 tools/api_census.py $out/adapt_trace > $out/adapt_census.txt 2>&1 || true
      python3 tools/idle_gaps.py $out/adapt_trace > $out/adapt_gaps.txt 2>&1 || true
      tail -n 40 $out/adapt_census.txt ;;
    adaptprof)
      # the 218k-leaf loop: plain timing, then a kernel + HIP-runtime trace and its census
      timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_plain.log 2>&1 || fail adapt_plain $? $out/adapt_plain.log
      tail -n 1 $out/adapt_plain.log
      timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/adapt_trace -o run -- python3 tools/adapt_loop.py > $out/adapt_trace.log 2>&1 || fail adapt_trace $? $out/adapt_trace.log
      python3 tools/api_census.py $out/adapt_trace > $out/adapt_census.txt 2>&1 || true
      head -n 30 $out/adapt_census.txt ;;
    adaptbigprof)
      # the 3.5 M-leaf loop: a kernel + HIP-runtime trace and its census
      ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/adapt_big_trace -o run -- python3 tools/adapt_loop.py > $out/adapt_big_trace.log 2>&1 || fail adapt_big_trace $? $out/adapt_big_trace.log
      python3 tools/api_census.py $out/adapt_big_trace > $out/adapt_big_census.txt 2>&1 || true
      head -n 30 $out/adapt_big_census.txt ;;
    adaptinc)
      # the 218k loop with the incremental list rebuild forced on, then off
      ADAPT_INCREMENTAL=1 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_inc1.log 2>&1 || fail adapt_inc1 $? $out/adapt_inc1.log
      tail -n 1 $out/adapt_inc1.log
      ADAPT_INCREMENTAL=0 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_inc0.log 2>&1 || fail adapt_inc0 $? $out/adapt_inc0.log
      tail -n 1 $out/adapt_inc0.log ;;
    adaptsplit)
      # adapt_grid in its parts (synchronised after each), at 218 k and 3.5 M
      # leaves, then the library's phase timers waiting for the device per lap
      ADAPT_SEG=2 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_split.log 2>&1 || fail adapt_split $? $out/adapt_split.log
      tail -n 3 $out/adapt_split.log
      ADAPT_SEG=2 ADAPT_N=1600 ADAPT_REL=0.006 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_big_split.log 2>&1 || fail adapt_big_split $? $out/adapt_big_split.log
      tail -n 3 $out/adapt_big_split.log
      ADAPT_N=1600 ADAPT_REL=0.006 DCCRGX_TIMING=2 timeout -k 10 300 python -u tools/adapt_loop.py > $out/adapt_big_sync_phases.log 2>&1 || fail adapt_sync_phases $? $out/adapt_big_sync_phases.log
      tail -n 2 $out/adapt_big_sync_phases.log ;;
    advlarge)
      timeout -k 10 300 python -u tools/run_adv_large.py > $out/adv_large.log 2>&1 || fail advlarge $? $out/adv_large.log
      tail -n 3 $out/adv_large.log ;;
    py=*)
      scr=${step#py=}; name=$(basename $scr .py)
      timeout -k 10 600 python -u $scr > $out/$name.log 2>&1 || fail $name $? $out/$name.log
      tail -n 5 $out/$name.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "pass $tag done"
