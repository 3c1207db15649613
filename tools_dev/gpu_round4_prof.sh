#!/bin/bash
# the trace and PMC half of tools_dev/gpu_round4.sh, as a gpurun call of its own
set -o pipefail
T=${1:-r04}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
bash tools_dev/gpu_trace.sh $T/trace || exit 4
bash tools_dev/gpu_pmc4.sh $T/pmc all || exit 5
echo done > gpurun_out/$T/rc_prof.txt
