#!/bin/bash
# Kernel-trace timelines of the stage bench (rocprofv3 --kernel-trace): the
# default 2-stream run and a 1-stream run of the same batches, for the busy-time
# union of the dominant kernel and the step's critical path
# (tools_dev/trace_busy.py).  usage (GPU box): bash tools_dev/gpu_trace.sh <tag> [extra bench args]
set -o pipefail
T=${1:-trace}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 20 --warmup 3 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s2 -o run --output-format csv -- python3 $B > $OUT/s2.json 2> $OUT/s2.err || { tail $OUT/s2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s1 -o run --output-format csv -- python3 $B --streams 1 > $OUT/s1.json 2> $OUT/s1.err || { tail $OUT/s1.err; exit 2; }
tail -c 600 $OUT/s2.json
echo done > $OUT/rc.txt
