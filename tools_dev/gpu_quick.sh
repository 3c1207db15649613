# quick GPU iteration: parity tests, then a short bench; usage: bash tools_dev/gpu_quick.sh <tag> [bench args]
set -o pipefail
TAG=${1:-q}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed" >> $OUT/gpu_tests.log; tail -30 $OUT/gpu_tests.log; exit 1; }
timeout -k 10 300 python bench.py --pairs 300000 --steps 10 --warmup 2 --no-cpu --no-host-path "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
