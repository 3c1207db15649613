#!/bin/bash
# side stream priority: low (4) vs normal (0); e2e stage with the sink stage
set -o pipefail
T=${1:-r5h}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for p in 4 0; do
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u tools_dev/regime_state_ab.py > $OUT/st$p.json 2> $OUT/st$p.err || { tail $OUT/st$p.err; exit 4; }
  echo "side $p" $(cat $OUT/st$p.json)
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path > $OUT/b$p.json 2> $OUT/b$p.err || { tail $OUT/b$p.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/b$p.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench side $p', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime --no-e2e --steps 4 > $OUT/e.json 2> $OUT/e.err || { tail $OUT/e.err; exit 3; }
python3 -c "
import json;d=json.load(open('$OUT/e.json'))
print('host_buffer_path', d.get('host_buffer_path',{}).get('value'))
print('end_to_end', json.dumps(d.get('end_to_end')))"
