#!/bin/bash
set -o pipefail
T=${1:-r5n}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), d.get('c5_refseed'), {k:v['ms_per_batch'] for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
