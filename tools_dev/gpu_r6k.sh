#!/bin/bash
# headline at 2 vs 3 caller streams (A/B, alternating)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6k
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for s in 2 3 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-seeding --no-regime --no-e2e --no-host-path --streams $s > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('streams $s', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
