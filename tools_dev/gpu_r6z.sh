#!/bin/bash
# caller streams 2 (default) vs 3 vs 4 on the stage bench, after the row bound
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6z
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for s in 2 3 2 3 2 3 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-host-path --no-regime --streams $s > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 5; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'))
print('$s', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline'].get('frac'))"
done
