#!/bin/bash
# stage-bench sweep: caller streams x extension workgroups per CU (same box)
set -o pipefail
T=${1:-sweep5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cfg in "2 2" "3 2" "2 1" "4 2" "2 2"; do
  set -- $cfg
  BWAGPU_EXT2_BLOCKS_PER_CU=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime --streams $1 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('streams $1 blocks/CU $2', d['value'], d['ms_per_step'], d['parity_all_steps'])"
done
