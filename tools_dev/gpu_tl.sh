# kernel-trace timelines of one reference-seeded batch: group kernels and wave-only
# usage (on the GPU box): bash tools_dev/gpu_tl.sh <tag>
set -o pipefail
TAG=${1:-tl}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
B="python3 $GRAFT_REPO_ROOT/tools_dev/realbench.py --batches 1 --reps 3"
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/g -o g --output-format csv -- $B > $OUT/g.log 2>&1 || { tail $OUT/g.log; exit 1; }
BWAGPU_EXT_WAVE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/w -o w --output-format csv -- $B > $OUT/w.log 2>&1 || { tail $OUT/w.log; exit 2; }
python3 $GRAFT_REPO_ROOT/tools_dev/timeline.py $OUT/g/g_kernel_trace.csv > $OUT/g.txt
python3 $GRAFT_REPO_ROOT/tools_dev/timeline.py $OUT/w/w_kernel_trace.csv > $OUT/w.txt
cat $OUT/g.txt $OUT/w.txt
