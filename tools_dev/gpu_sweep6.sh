#!/bin/bash
# stage bench + regime legs: extension workgroups per CU 1 vs 2, alternating (same box)
set -o pipefail
T=${1:-sweep6}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 1 2 3; do
for bl in 1 2; do
  BWAGPU_EXT2_BLOCKS_PER_CU=$bl timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('blocks/CU $bl', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'], {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
done
