# spec path quick check: parity (spec param + C2 reference-seeded), realbench, selection trace
set -o pipefail
TAG=${1:-spec}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spec or not c2a_path" > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/real150.json 2> $OUT/real150.err || { tail $OUT/real150.err; exit 2; }
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 --length mix --pairs 24000 > $OUT/realmix.json 2> $OUT/realmix.err || { tail $OUT/realmix.err; exit 3; }
cat $OUT/real150.json $OUT/realmix.json
timeout -k 10 200 python -u tools_dev/spec_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 4; }
cat $OUT/trace.json
