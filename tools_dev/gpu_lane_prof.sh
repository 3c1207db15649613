#!/bin/bash
# rocprofv3 kernel summary of the stage bench with the lane kernel on (mode $LM)
set -o pipefail
T=${1:-laneprof}
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/$T
cd /tmp && BWAGPU_EXT_LANE=${LM:-2} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$T/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/$T/prof.log 2>&1 || exit 3
head -14 $GRAFT_REPO_ROOT/gpurun_out/$T/prof/run_kernel_stats.csv | cut -c1-100,200-300
