#!/bin/bash
set -o pipefail
T=${1:-g4b}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "chain_sets or ksw_extend2" tests/test_gpu_c2_batch.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for g in 1 2 3 1 2 3; do
BWAGPU_EXT2_BLOCKS_PER_CU=$g timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-regime --no-seeding > $OUT/b$g.json 2> $OUT/b$g.err || { tail $OUT/b$g.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/b$g.json'));r=d['roofline'];print('grid',$g,d['value'],d['ms_per_step'],d['parity_all_steps'],{k:r[k] for k in ('kernel_ms_per_step','frac','frac_isolated','isolated_launch_ms')})"
done
