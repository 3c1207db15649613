#!/bin/bash
# regime leg A/B: counters / HIP events, and the bench's own regime_stage
set -o pipefail
T=${1:-r5b}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in "" "--stats" "--prof" "--stats --prof"; do
  timeout -k 10 300 python -u tools_dev/regime_ab.py --modes c2b0,c3r $f > $OUT/ab.json 2> $OUT/ab.err || { tail $OUT/ab.err; exit 2; }
  echo "flags [$f]" $(cat $OUT/ab.json)
done
timeout -k 10 300 python -u -c "
import sys, json, torch; sys.argv=['bench.py']
import bench
dev=torch.device('cuda:0')
r=bench.regime_stage(dev)
print(json.dumps({k:v.get('ms_per_batch') for k,v in r.items() if isinstance(v,dict)}))
" > $OUT/rs.json 2> $OUT/rs.err || { tail $OUT/rs.err; exit 3; }
cat $OUT/rs.json
