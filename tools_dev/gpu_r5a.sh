#!/bin/bash
# Round-5 first call: the stage bench on this tree, the regime A/B
# (tools_dev/regime_ab.py) and kernel traces of its three main patterns.
set -o pipefail
T=${1:-r5a}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));g=d.get('regime_grch38',{});r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r.get('kernel_ms_per_step'), {k:v['ms_per_batch'] for k,v in g.items() if isinstance(v,dict) and 'ms_per_batch' in v})"
timeout -k 10 400 python -u tools_dev/regime_ab.py > $OUT/ab.json 2> $OUT/ab.err || { tail $OUT/ab.err; exit 2; }
cat $OUT/ab.json
cd /tmp
for m in c2alt c2b0 c3r; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_dev/regime_ab.py --modes $m > $OUT/tr_$m.json 2> $OUT/tr_$m.err || { tail $OUT/tr_$m.err; exit 3; }
done
echo done > $OUT/rc.txt
