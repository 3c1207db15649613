set -o pipefail
TAG=${1:-tl2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/b -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --streams 1 --steps 10 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/r -o r --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 2 --reps 3 > $OUT/r.log 2>&1 || { tail $OUT/r.log; exit 2; }
python3 $GRAFT_REPO_ROOT/tools_dev/timeline.py $OUT/b/b_kernel_trace.csv > $OUT/b.txt
python3 $GRAFT_REPO_ROOT/tools_dev/timeline.py $OUT/r/r_kernel_trace.csv > $OUT/r.txt
ls $OUT/b $OUT/r
cat $OUT/b.txt $OUT/r.txt
