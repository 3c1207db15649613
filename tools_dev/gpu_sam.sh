# SAM parity on the GPU box + the kernel A/B after the queue-head change
# usage: bash tools_dev/gpu_sam.sh <tag>
set -o pipefail
TAG=${1:-sam}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sam_parity.py tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/real150.json 2> $OUT/real150.err || { tail $OUT/real150.err; exit 2; }
cat $OUT/real150.json
timeout -k 10 300 python bench.py --no-cpu --no-cigar > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
cat $OUT/bench.json
