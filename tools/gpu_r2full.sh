# full GPU suite, then the default bench line: $1 = tag
set -u
TAG=${1:-full}
bash tools/gpu_tests.sh $TAG && bash tools/gpu_bench.sh $TAG
