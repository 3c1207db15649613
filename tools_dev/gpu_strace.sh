#!/bin/bash
# per-read selection trace of one reference-seeded C2 batch (tools_dev/spec_trace.py)
set -o pipefail
T=${1:-strace}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools_dev/spec_trace.py > $OUT/trace.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/trace.json'))
for p in d:
  print(p, d[p]['span_us'])
  for s in ('light','heavy','heavy_mat'):
    if s in d[p]: print('  ',s,{k:v for k,v in d[p][s].items() if k!='slowest'}, d[p][s]['slowest'][:3])
  print('  in_flight', d[p]['in_flight'])"
