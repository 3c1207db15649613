#!/bin/bash
# quad-kernel grid A/B (workgroups per CU), stage bench only
set -o pipefail
T=${1:-g4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for g in ${GRIDS:-2 3 2 3}; do
BWAGPU_EXT2_BLOCKS_PER_CU=$g timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/b$g.json 2> $OUT/b$g.err || { tail $OUT/b$g.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/b$g.json'));r=d['roofline'];print('grid',$g,d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','frac','frac_isolated','isolated_launch_ms')})"
done
