#!/bin/bash
# PMC passes of the stage bench (one rocprofv3 --pmc run per counter group):
# SQ issue/wait/LDS counters, then FETCH_SIZE and WRITE_SIZE each alone.
# Summaries: tools_dev/pmc_round.py (per-sequence counters, lane-ops per
# algorithmic cell) and tools_dev/pmc_traffic.py (HBM bytes per launch).
# usage (GPU box): bash tools_dev/gpu_pmc4.sh <tag> [sq|all] [extra bench args]
set -o pipefail
T=${1:-pmc4}; W=${2:-all}; shift; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding --steps 5 --warmup 1 $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_a -o a --output-format csv -- python3 $B > $OUT/a.json 2> $OUT/a.err || { tail $OUT/a.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_b -o b --output-format csv -- python3 $B > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 2; }
if [ "$W" = all ]; then
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 $B > $OUT/f.json 2> $OUT/f.err || { tail $OUT/f.err; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 $B > $OUT/w.json 2> $OUT/w.err || { tail $OUT/w.err; exit 4; }
fi
cd $GRAFT_REPO_ROOT
python3 tools_dev/pmc_round.py $OUT $OUT/a.json > $OUT/summary.json && cat $OUT/summary.json
echo done > $OUT/rc.txt
