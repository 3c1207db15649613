# A/B of the extension kernels on reference-seeded batches: parity tests, then
# realbench with the group kernels (default) and with BWAGPU_EXT_WAVE=1.
# usage (on the GPU box): bash tools_dev/gpu_ab_ext.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-ab}; SKIPT=${2:-0}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ "$SKIPT" != "1" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2_batch.py tests/test_host_stage.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
fi
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/grp.json 2> $OUT/grp.err || { tail $OUT/grp.err; exit 2; }
BWAGPU_EXT_WAVE=1 timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 > $OUT/wave.json 2> $OUT/wave.err || { tail $OUT/wave.err; exit 3; }
timeout -k 10 200 python -u tools_dev/realbench.py --batches 2 --reps 10 --length mix --pairs 24000 > $OUT/grpmix.json 2> $OUT/grpmix.err || { tail $OUT/grpmix.err; exit 4; }
cat $OUT/grp.json $OUT/wave.json $OUT/grpmix.json
