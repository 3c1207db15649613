#!/bin/bash
# row bound check period: every row (p0), 2 (p1), 4 (default), 8 (p7)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6y
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for v in def p1 p7 p0 def p1 p7 p0; do
  L=""; [ $v != def ] && L="BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/lib_$v/libbwagpu.so"
  env $L timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));c=d.get('c5_refseed',{})
print('$v', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline'].get('frac'), c.get('ms_per_batch'), c.get('parity_all_steps'), {k:(v['ms_per_batch'], v['parity_all_steps']) for k,v in d.get('regime_grch38',{}).items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
