#!/bin/bash
# SQ counters of the dominant extension kernel with and without the
# two-seeds-per-wave path (BWAGPU_EXT_PAIR), two counter groups per setting.
set -o pipefail
T=${1:-pairpmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-cigar --no-host-path --no-seeding --no-regime --steps 8 --warmup 1"
for p in ${MODES:-0 2}; do
  export BWAGPU_EXT_PAIR=$p
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/a$p -o a --output-format csv -- $B > $OUT/a$p.log 2>&1 || { tail $OUT/a$p.log; exit 4; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $OUT/b$p -o b --output-format csv -- $B > $OUT/b$p.log 2>&1 || { tail $OUT/b$p.log; exit 5; }
done
echo done > $OUT/rc.txt
