#!/bin/bash
# Round 6's profiles of one tree (a gpurun call of its own): kernel traces of
# the headline (3 caller streams and 1), the SQ and FETCH/WRITE PMC passes,
# and a kernel trace of the whole default bench in the driver's leg order
# (--steps 20 --warmup 5) for the regime legs.  Summaries afterwards:
# tools_dev/trace_busy.py, pmc_round.py, pmc_traffic.py (workload c2_stream).
# usage (GPU box): bash tools_dev/gpu_round6_prof.sh <tag> [nofull]
set -o pipefail
T=${1:-r06}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
bash tools_dev/gpu_trace.sh $T/trace --headline-only --stream-batches 24 || exit 4
bash tools_dev/gpu_pmc4.sh $T/pmc all --headline-only --stream-batches 8 || exit 5
if [ "$2" != nofull ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/full -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $OUT/full.json 2> $OUT/full.err || { tail $OUT/full.err; exit 6; }
fi
echo done > $OUT/rc_prof.txt
