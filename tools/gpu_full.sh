#!/bin/bash
# Round-end style GPU pass: every -m gpu test, smoke, the bench line, and the
# rocprofv3 kernel-trace + separate FETCH_SIZE / WRITE_SIZE passes of the
# headline bench that tools/summarize_prof.py turns into profiles/<tag>_summary.json.
# usage (through gpurun): bash tools/gpu_full.sh <tag> [skip-tests|tests] [noprof]
set -o pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 || { tail -n 40 $out/gpu_tests.log; exit 1; }
  tail -n 2 $out/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 \
    || { tail -n 20 $out/smoke.log; exit 1; }
fi
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || { tail -n 20 $out/bench.log; exit 1; }
tail -n 1 $out/bench.log
[ "$3" = "noprof" ] && { echo done; exit 0; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof/trace -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-secondary --no-halo-payload --no-cpu-baseline --no-check \
  > $out/prof_trace.log 2>&1 || { tail -n 20 $out/prof_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/prof/fetch -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-secondary --no-halo-payload --no-cpu-baseline --no-check \
  > $out/prof_fetch.log 2>&1 || { tail -n 20 $out/prof_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/prof/write -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-secondary --no-halo-payload --no-cpu-baseline --no-check \
  > $out/prof_write.log 2>&1 || { tail -n 20 $out/prof_write.log; exit 1; }
find $out/prof -name '*.csv' | head -n 20
echo done
