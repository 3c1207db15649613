#!/bin/bash
set -o pipefail
T=${1:-r5s}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for q in 8 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b$q.json 2> $OUT/b$q.err || { tail $OUT/b$q.err; exit 5; }
python3 -c "
import json;d=json.load(open('$OUT/b$q.json'));r=d['roofline'];c=d.get('c5_refseed',{})
print('queues $q bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), c.get('ms_per_batch'), c.get('parity_all_steps'), {k:v['ms_per_batch'] for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools_dev/e2e_ab.py 2 3 4 > $OUT/e.json 2> $OUT/e.err || { tail $OUT/e.err; exit 1; }
cat $OUT/e.json
