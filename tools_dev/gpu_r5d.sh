#!/bin/bash
# side-stream priority A/B on the regime-state tool and the bench's regime leg
set -o pipefail
T=${1:-r5d}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for p in ${PRIOS:-0 1}; do
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u tools_dev/regime_state_ab.py > $OUT/st$p.json 2> $OUT/st$p.err || { tail $OUT/st$p.err; exit 2; }
  echo "prio $p" $(cat $OUT/st$p.json)
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding > $OUT/b$p.json 2> $OUT/b$p.err || { tail $OUT/b$p.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/b$p.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench prio $p', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
done
cd /tmp
BWAGPU_SIDE_PRIO=${TRP:-0} timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr0 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/regime_state_ab.py > $OUT/tr0.json 2> $OUT/tr0.err || { tail $OUT/tr0.err; exit 3; }
