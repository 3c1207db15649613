# Full GPU check: every -m gpu test, then realbench on reference-seeded batches (150 bp, mixed).
# usage (on the GPU box): bash tools_dev/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-check}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/real150.json 2> $OUT/real150.err || { tail $OUT/real150.err; exit 2; }
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 --length mix --pairs 24000 > $OUT/realmix.json 2> $OUT/realmix.err || { tail $OUT/realmix.err; exit 3; }
cat $OUT/real150.json $OUT/realmix.json
