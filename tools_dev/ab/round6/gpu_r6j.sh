#!/bin/bash
# round 6: kernel traces (3 / 1 caller streams) and SQ PMC passes of the
# headline (stream workload), phased tree — where the step goes
set -o pipefail
T=${1:-r06j}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
bash tools_dev/gpu_trace.sh $T/trace --headline-only --stream-batches 24 || exit 4
bash tools_dev/gpu_pmc4.sh $T/pmc sq --headline-only --stream-batches 8 || exit 5
cd $GRAFT_REPO_ROOT
python3 tools_dev/trace_busy.py $OUT/trace/s2/run_kernel_trace.csv 3 20 "spec_side4_kernel<16, 10, true>" > $OUT/busy3.json
python3 tools_dev/trace_busy.py $OUT/trace/s1/run_kernel_trace.csv 3 20 "spec_side4_kernel<16, 10, true>" > $OUT/busy1.json
head -c 1500 $OUT/busy3.json
echo done > $OUT/rc.txt
