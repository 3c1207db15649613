# SAM stage on the device (gpusam mode of oracle/_ref/sam_harness): one direct
# run with its timings, then the SAM parity tests
# usage: bash tools_dev/gpu_samstage.sh <tag>
set -o pipefail
TAG=${1:-samstage}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/w
timeout -k 10 120 oracle/_ref/sam_harness ${MODE:-gpusam} $OUT/w $OUT/w/gpusam.sam 7 10000 150 10000000 8 > $OUT/direct.log 2>&1 || { echo "direct run failed: $?" >> $OUT/direct.log; tail -20 $OUT/direct.log; exit 1; }
tail -2 $OUT/direct.log
timeout -k 10 120 oracle/_ref/sam_harness ref $OUT/w $OUT/w/ref.sam 7 10000 150 10000000 8 > $OUT/ref.log 2>&1 || { tail -5 $OUT/ref.log; exit 2; }
tail -1 $OUT/ref.log
cmp $OUT/w/ref.sam $OUT/w/gpusam.sam && echo SAM_IDENTICAL
rm -f $OUT/w/*.sam $OUT/w/ref.fa*
timeout -k 10 600 python -u -m pytest tests/test_sam_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "pytest failed" >> $OUT/tests.log; tail -40 $OUT/tests.log; exit 3; }
tail -3 $OUT/tests.log
