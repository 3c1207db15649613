#!/bin/bash
set -o pipefail
T=${1:-r5t}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ns in 2 3 4 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime --streams $ns > $OUT/bs$ns.json 2> $OUT/bs$ns.err || { tail $OUT/bs$ns.err; exit 7; }
  python3 -c "
import json;d=json.load(open('$OUT/bs$ns.json'));r=d['roofline']
print('streams $ns', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
