set -o pipefail
TAG=${1:-tl3}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/b -o b --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --streams 1 --steps 10 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools_dev/timeline.py $OUT/b/b_kernel_trace.csv > $OUT/b.txt
cat $OUT/b.txt
